"""RandLA-Net on MI355X (reference
ml3d/torch/models/randlanet.py).

``RandLANet`` keeps the reference module tree — the same submodule names,
classes and parameter shapes, so a reference ``state_dict`` (270 entries,
1,242,307 trainable parameters) loads unchanged — but runs channels-last:
per-point tensors [N, C], per-neighbour tensors [N, K, C], the 1x1
convolutions as GEMMs, BatchNorm folded into them at inference, and the
index work (neighbour relative encoding, attentive-pooling softmax/sum,
random-sample max pooling) in HIP kernels (csrc/randla.hip).  The
differentiable path (training / autograd) uses the same layout with torch
ops.

``SemSegInference`` is the GPU counterpart of
``SemanticSegmentation.run_inference`` with the
``SemSegSpatiallyRegularSampler`` patch loop (semantic_segmentation.py:122-180,
semseg_spatially_regular.py:62-111, randlanet.py:115-239, 441-465): the cloud
is grid-subsampled and projected ONCE, then patches are cropped, recentred,
searched (kNN k=16 / k=1 per layer), inferred and accumulated on the GPU
until every sub-point's possibility exceeds 0.5.
"""
import itertools
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from ._util import metric_code, ptr, stream_handle

_BN_EPS = 1e-6


# ---------------------------------------------------------------------------
# HIP kernels (csrc/randla.hip)
# ---------------------------------------------------------------------------
def relative_encoding(coords, nbr):
    """[N,3] f32, [N,K] int32 -> [N,K,10]: (|c-p|, c-p, c, p) (randlanet.py:593-606)."""
    n, k = nbr.shape
    out = torch.empty((n, k, 10), dtype=torch.float32, device=coords.device)
    _lib.call("o3dml_randla_relative_encoding", ptr(coords), n, ptr(nbr), k, ptr(out), stream_handle(coords.device))
    return out


def attentive_pool(x, logits):
    """softmax over K of logits, weighted sum of x: [N,K,C] x2 -> [N,C] (randlanet.py:632-650)."""
    n, k, c = x.shape
    out = torch.empty((n, c), dtype=torch.float32, device=x.device)
    _lib.call("o3dml_randla_attentive_pool", ptr(x), ptr(logits), n, k, c, ptr(out), stream_handle(x.device))
    return out


def gather_max(feat, idx):
    """out[m] = max_k feat[idx[m, k]]: [N,C], [M,K] int32 -> [M,C] (randlanet.py:306-331)."""
    m, k = idx.shape
    c = feat.shape[1]
    out = torch.empty((m, c), dtype=torch.float32, device=feat.device)
    _lib.call("o3dml_randla_gather_max", ptr(feat), c, ptr(idx), m, k, ptr(out), stream_handle(feat.device))
    return out


def concat_rows(a, ia, b, ib):
    """[a[ia] | b[ib]] row-wise (ia / ib None = identity), channels-last:
    a [Na, da], b [Nb, db] -> [rows, da + db]; rows = len(ia) or len(a)."""
    rows = ia.numel() if ia is not None else a.shape[0]
    da, db = a.shape[-1], b.shape[-1]
    out = torch.empty((rows, da + db), dtype=torch.float32, device=a.device)
    _lib.call("o3dml_concat_rows", ptr(a), da, ptr(ia), 64 if ia is not None and ia.dtype == torch.int64 else 32,
              ptr(b), db, ptr(ib), 64 if ib is not None and ib.dtype == torch.int64 else 32, rows, ptr(out),
              stream_handle(a.device))
    return out


def dense_act(a1, w, b, slope=None, a2=None, a2_index=None):
    """act([a1 | a2[a2_index]] @ w^T + b) in one launch (csrc/dense.hip):
    a1 [N, k1] (or None: k1 = 0), a2 [*, k2] (rows selected by a2_index int64
    [N], or a2 [N, k2] itself), w [M, k1 + k2], b [M]; act = LeakyReLU(slope),
    none if slope is None."""
    if a1 is None:  # only the gathered operand: rows a2[a2_index] (or a2 itself)
        n, k1 = (a2_index.shape[0] if a2_index is not None else a2.shape[0]), 0
    else:
        n, k1 = a1.shape
    k2 = 0 if a2 is None else a2.shape[1]
    m = w.shape[0]
    dev = (a1 if a1 is not None else a2).device
    out = torch.empty((n, m), dtype=torch.float32, device=dev)
    nbytes = _lib.load().o3dml_dense_act_workspace_size(n, k1 + k2, m)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev) if nbytes else None
    # operands bound to names: a temporary freed inside the argument list could
    # be handed to the next temporary by the caching allocator before the launch
    a1 = None if a1 is None else a1.contiguous()
    a2 = None if a2 is None else a2.contiguous()
    _lib.call("o3dml_dense_act", ptr(a1), k1, ptr(a2), k2,
              ptr(a2_index), ptr(w), ptr(b), n, m, int(slope is not None), float(slope or 0.0), ptr(out), ptr(ws),
              0 if ws is None else ws.numel(), stream_handle(dev))
    return out


def _fused():
    return not torch.is_grad_enabled()


# ---------------------------------------------------------------------------
# modules (same names / parameters as the reference)
# ---------------------------------------------------------------------------
class SharedMLP(nn.Module):
    """1x1 Conv2d / ConvTranspose2d + BatchNorm2d + activation (randlanet.py:469-512),
    applied to channels-last rows."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, transpose=False, bn=True,
                 activation_fn=None):
        super().__init__()
        conv = nn.ConvTranspose2d if transpose else nn.Conv2d
        self.conv = conv(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                         padding=(kernel_size - 1) // 2)
        self.transpose = transpose
        self.batch_norm = nn.BatchNorm2d(out_channels, eps=_BN_EPS, momentum=0.01) if bn else None
        self.activation_fn = activation_fn
        self._folded = None

    def _weight(self):
        w = self.conv.weight[:, :, 0, 0]
        return w.t() if self.transpose else w  # [out, in]

    def folded(self):
        """(W [out,in], b [out]) with eval-mode BatchNorm folded in."""
        if self._folded is None:
            with torch.no_grad():
                w, b = self._weight().float(), self.conv.bias.float()
                if self.batch_norm is not None:
                    bn = self.batch_norm
                    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
                    w = w * scale[:, None]
                    b = (b - bn.running_mean) * scale + bn.bias
                self._folded = (w.contiguous(), b.contiguous())
        return self._folded

    def slope(self):
        """LeakyReLU slope of the activation, None without one (eval fused path)."""
        a = self.activation_fn
        return None if a is None else (a.negative_slope if isinstance(a, nn.LeakyReLU) else False)

    def forward(self, x):
        """x [..., in] -> [..., out]."""
        if _fused() and not self.training and self.slope() is not False:
            w, b = self.folded()  # BN folded; bias + LeakyReLU in the GEMM epilogue (csrc/dense.hip)
            y = dense_act(x.reshape(-1, x.shape[-1]), w, b, self.slope())
            return y.reshape(*x.shape[:-1], w.shape[0])
        if _fused() and not self.training:
            w, b = self.folded()
            y = torch.addmm(b, x.reshape(-1, x.shape[-1]), w.t()).reshape(*x.shape[:-1], w.shape[0])
        else:
            y = F.linear(x, self._weight(), self.conv.bias)
            if self.batch_norm is not None:
                bn = self.batch_norm
                y = F.batch_norm(y.reshape(-1, y.shape[-1]), bn.running_mean, bn.running_var, bn.weight, bn.bias,
                                 self.training, bn.momentum, bn.eps).reshape(y.shape)
        if self.activation_fn is not None:
            y = self.activation_fn(y)
        return y


class LocalSpatialEncoding(nn.Module):
    """randlanet.py:540-606."""

    def __init__(self, dim_in, dim_out, num_neighbors, encode_pos=False):
        super().__init__()
        self.num_neighbors = num_neighbors
        self.mlp = SharedMLP(dim_in, dim_out, activation_fn=nn.LeakyReLU(0.2))
        self.encode_pos = encode_pos

    def forward(self, coords, features, nbr, relative_features=None):
        """coords [N,3], features [N,d], nbr [N,K] int32 -> ([N,K,d+dout], relative [N,K,dout])."""
        n, k = nbr.shape
        if self.encode_pos:
            if _fused():
                rel = relative_encoding(coords, nbr)
            else:
                nc = coords[nbr.long()]
                ext = coords[:, None, :].expand(n, k, 3)
                rp = ext - nc
                rel = torch.cat([torch.sqrt((rp * rp).sum(-1, keepdim=True)), rp, ext, nc], -1)
            relative_features = rel
        elif relative_features is None:
            raise ValueError("LocalSpatialEncoding: Require relative_features for second pass.")
        relative_features = self.mlp(relative_features)
        if _fused():
            cat = concat_rows(features.contiguous(), nbr.reshape(-1), relative_features.contiguous(), None)
            return cat.view(n, k, -1), relative_features
        neighbor_features = features[nbr.long()]
        return torch.cat([neighbor_features, relative_features], -1), relative_features


class AttentivePooling(nn.Module):
    """randlanet.py:609-650."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.score_fn = nn.Sequential(nn.Linear(in_channels, in_channels), nn.Softmax(dim=-2))
        self.mlp = SharedMLP(in_channels, out_channels, activation_fn=nn.LeakyReLU(0.2))

    def forward(self, x):
        """x [N,K,C] -> [N,Cout]."""
        lin = self.score_fn[0]
        logits = F.linear(x, lin.weight, lin.bias)
        if _fused():
            pooled = attentive_pool(x.contiguous(), logits.contiguous())
        else:
            pooled = (torch.softmax(logits, dim=-2) * x).sum(-2)
        return self.mlp(pooled)


class LocalFeatureAggregation(nn.Module):
    """randlanet.py:653-692."""

    def __init__(self, d_in, d_out, num_neighbors):
        super().__init__()
        self.num_neighbors = num_neighbors
        self.mlp1 = SharedMLP(d_in, d_out // 2, activation_fn=nn.LeakyReLU(0.2))
        self.lse1 = LocalSpatialEncoding(10, d_out // 2, num_neighbors, encode_pos=True)
        self.pool1 = AttentivePooling(d_out, d_out // 2)
        self.lse2 = LocalSpatialEncoding(d_out // 2, d_out // 2, num_neighbors)
        self.pool2 = AttentivePooling(d_out, d_out)
        self.mlp2 = SharedMLP(d_out, 2 * d_out)
        self.shortcut = SharedMLP(d_in, 2 * d_out)
        self.lrelu = nn.LeakyReLU()

    _ATT_WIDTHS = (16, 32, 64, 128, 256)

    def _att_weights(self, lse, pool):
        """(Wr^T, br, Ws^T, bs) for the fused kernel, cached until parameters change."""
        cache = self.__dict__.setdefault("_t_cache", {})
        key = id(pool)
        if key not in cache:
            with torch.no_grad():
                wr, br = lse.mlp.folded()
                lin = pool.score_fn[0]
                cache[key] = (wr.t().contiguous(), br.contiguous(), lin.weight.float().t().contiguous(),
                              lin.bias.float().contiguous())
        return cache[key]

    def _fused_pool(self, coords, x, nbr, lse, pool, rel_in):
        """LocalSpatialEncoding + AttentivePooling in one HIP pass
        (csrc/randla.hip att_pool_kernel) -> (pooled [N, d], rel [N, K, d/2])."""
        n, k = nbr.shape
        d = pool.score_fn[0].weight.shape[0]
        wrt, br, wst, bs = self._att_weights(lse, pool)
        out = torch.empty((n, d), dtype=torch.float32, device=x.device)
        rel = torch.empty((n, k, d // 2), dtype=torch.float32, device=x.device) if rel_in is None else None
        _lib.call("o3dml_randla_att_pool", ptr(coords), ptr(x.contiguous()), ptr(nbr), n, k, d,
                  ptr(rel_in), ptr(wrt), ptr(br), ptr(wst), ptr(bs), ptr(rel), ptr(out), stream_handle(x.device))
        return out, rel

    def _tail_weights(self):
        """lrelu(mlp2(x) + shortcut(feat)) as ONE GEMM over [x | feat]:
        ([W2 | Ws], b2 + bs), BatchNorms folded; cached like _att_weights."""
        cache = self.__dict__.setdefault("_t_cache", {})
        if "tail" not in cache:
            with torch.no_grad():
                w2, b2 = self.mlp2.folded()
                ws, bs = self.shortcut.folded()
                cache["tail"] = (torch.cat([w2, ws], 1).contiguous(), (b2 + bs).contiguous())
        return cache["tail"]

    def forward(self, coords, feat, nbr):
        x = self.mlp1(feat)
        d = self.pool1.score_fn[0].weight.shape[0]
        if (_fused() and not self.training and nbr.shape[1] == 16 and d in self._ATT_WIDTHS
                and nbr.dtype == torch.int32):
            pooled, rel = self._fused_pool(coords.contiguous(), x, nbr.contiguous(), self.lse1, self.pool1, None)
            x = self.pool1.mlp(pooled)
            pooled, _ = self._fused_pool(coords.contiguous(), x, nbr.contiguous(), self.lse2, self.pool2, rel)
            x = self.pool2.mlp(pooled)
            w, b = self._tail_weights()
            return dense_act(x, w, b, self.lrelu.negative_slope, a2=feat)
        x, rel = self.lse1(coords, x, nbr)
        x = self.pool1(x)
        x, _ = self.lse2(coords, x, nbr, relative_features=rel)
        x = self.pool2(x)
        return self.lrelu(self.mlp2(x) + self.shortcut(feat))


class RandLANet(nn.Module):
    """Module tree and state_dict of ml3d RandLANet (randlanet.py:16-113);
    forward takes the reference ``inputs`` dict ([B, N, ...] lists) and returns
    [B, N, num_classes] scores."""

    def __init__(self, name="RandLANet", num_neighbors=16, num_layers=4, num_points=4096 * 11, num_classes=19,
                 ignored_label_inds=(0,), sub_sampling_ratio=(4, 4, 4, 4), in_channels=3, dim_features=8,
                 dim_output=(16, 64, 128, 256), grid_size=0.06, **kwargs):
        super().__init__()
        self.cfg = dict(name=name, num_neighbors=num_neighbors, num_layers=num_layers, num_points=num_points,
                        num_classes=num_classes, ignored_label_inds=list(ignored_label_inds),
                        sub_sampling_ratio=list(sub_sampling_ratio), in_channels=in_channels,
                        dim_features=dim_features, dim_output=list(dim_output), grid_size=grid_size, **kwargs)
        self.fc0 = nn.Linear(in_channels, dim_features)
        self.bn0 = nn.BatchNorm2d(dim_features, eps=_BN_EPS, momentum=0.01)
        encoder, enc_dims = [], []
        d = dim_features
        for i in range(num_layers):
            encoder.append(LocalFeatureAggregation(d, dim_output[i], num_neighbors))
            d = 2 * dim_output[i]
            if i == 0:
                enc_dims.append(d)
            enc_dims.append(d)
        self.encoder = nn.ModuleList(encoder)
        self.mlp = SharedMLP(d, d, activation_fn=nn.LeakyReLU(0.2))
        decoder = []
        for i in range(num_layers):
            decoder.append(SharedMLP(enc_dims[-i - 2] + d, enc_dims[-i - 2], transpose=True,
                                     activation_fn=nn.LeakyReLU(0.2)))
            d = enc_dims[-i - 2]
        self.decoder = nn.ModuleList(decoder)
        self.fc1 = nn.Sequential(SharedMLP(d, 64, activation_fn=nn.LeakyReLU(0.2)),
                                 SharedMLP(64, 32, activation_fn=nn.LeakyReLU(0.2)), nn.Dropout(0.5),
                                 SharedMLP(32, num_classes, bn=False))

    def _fc0_folded(self):
        """fc0 with eval-mode bn0 folded in (randlanet.py:262-265)."""
        if getattr(self, "_fc0_cache", None) is None:
            with torch.no_grad():
                bn = self.bn0
                scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
                w = (self.fc0.weight * scale[:, None]).float().contiguous()
                b = ((self.fc0.bias - bn.running_mean) * scale + bn.bias).float().contiguous()
                self._fc0_cache = (w, b)
        return self._fc0_cache

    # folded eval weights are invalidated whenever parameters may change; the
    # captured patch graphs hold raw pointers to them, so they go too
    def _invalidate(self):
        self._fc0_cache = None
        for m in self.modules():
            if isinstance(m, SharedMLP):
                m._folded = None
            if isinstance(m, LocalFeatureAggregation):
                m.__dict__.pop("_t_cache", None)
        self.__dict__.pop("_o3dml_patch_step", None)
        self.__dict__.pop("_o3dml_patch_graph", None)

    def train(self, mode=True):
        # eval() on a model already in eval mode keeps the folded weights and
        # the graphs built on them (SemSegInference.run calls it per frame)
        if mode or self.training:
            self._invalidate()
        return super().train(mode)

    def load_state_dict(self, *a, **kw):
        self._invalidate()
        return super().load_state_dict(*a, **kw)

    def _apply(self, fn, *a, **kw):
        # .to() / .half() / .cuda() replace the parameters: the folded copies
        # (and graphs on them) would keep the old values
        self._invalidate()
        return super()._apply(fn, *a, **kw)

    def _sync_folded(self):
        """Drop the folded eval weights (and the graphs built on them) if any
        parameter or buffer was modified in place since they were made (an
        in-place copy_, an optimizer step in eval mode): the tensors' version
        counters are compared, once per frame / forward call."""
        v = tuple(t._version for t in itertools.chain(self.parameters(), self.buffers()))
        if self.__dict__.get("_o3dml_wver") != v:
            self._invalidate()
            self.__dict__["_o3dml_wver"] = v

    def forward_points(self, feat, coords, nbrs, subs, ups):
        """One or more concatenated patches, channels-last.
        feat [N0,Cin]; coords[i] [Ni,3]; nbrs[i] [Ni,K] int32; subs[i] [N(i+1),K] int32
        (indices into level i); ups[i] [Ni] int64 (indices into level i+1).
        Returns logits [N0, num_classes]."""
        bn = self.bn0
        if _fused() and not self.training:
            w, b = self._fc0_folded()
            x = dense_act(feat, w, b, 0.2)
        else:
            x = F.linear(feat, self.fc0.weight, self.fc0.bias)
            x = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, self.training, bn.momentum,
                             bn.eps)
            x = F.leaky_relu(x, 0.2)
        enc = []
        for i, layer in enumerate(self.encoder):
            y = layer(coords[i], x, nbrs[i])
            if _fused():
                ys = gather_max(y.contiguous(), subs[i])
            else:
                ys = y[subs[i].long()].max(1).values
            if i == 0:
                enc.append(y)
            enc.append(ys)
            x = ys
        x = self.mlp(x)
        for i, layer in enumerate(self.decoder):
            if _fused() and not self.training:  # [skip | upsampled] gathered inside the GEMM
                w, b = layer.folded()
                x = dense_act(enc[-i - 2], w, b, layer.slope(), a2=x, a2_index=ups[-i - 1])
            elif _fused():
                x = layer(concat_rows(enc[-i - 2].contiguous(), None, x.contiguous(), ups[-i - 1]))
            else:
                x = layer(torch.cat([enc[-i - 2], x[ups[-i - 1]]], -1))
        for m in self.fc1:
            x = m(x)
        return x

    def forward(self, inputs):
        """Reference signature (randlanet.py:241-298): inputs['features'] [B,N,Cin],
        'coords'/'neighbor_indices'/'sub_idx'/'interp_idx' lists of [B,...]."""
        dev = next(self.parameters()).device
        self._sync_folded()
        feats = inputs["features"].to(dev).float()
        B, N, _ = feats.shape
        L = len(self.encoder)
        coords, nbrs, subs, ups = [], [], [], []
        for i in range(L):
            c = inputs["coords"][i].to(dev).float()
            ni = c.shape[1]
            off = (torch.arange(B, device=dev) * ni).view(B, 1, 1)
            nb = inputs["neighbor_indices"][i].to(dev).long()
            coords.append(c.reshape(-1, 3).contiguous())
            nbrs.append((nb + off).reshape(-1, nb.shape[-1]).int().contiguous())
            sb = inputs["sub_idx"][i].to(dev).long()
            subs.append((sb + off).reshape(-1, sb.shape[-1]).int().contiguous())
            up = inputs["interp_idx"][i].to(dev).long().reshape(B, -1)
            n_next = inputs["coords"][i + 1].shape[1] if i + 1 < L else sb.shape[1]
            ups.append((up + (torch.arange(B, device=dev) * n_next).view(B, 1)).reshape(-1))
        out = self.forward_points(feats.reshape(B * N, -1).contiguous(), coords, nbrs, subs, ups)
        return out.reshape(B, N, -1)


# ---------------------------------------------------------------------------
# inference pipeline (GPU)
# ---------------------------------------------------------------------------
def up_from_knn(nb_all, cat, rs, nxt, srs, scratch=None):
    """Up-sampling indices of the RandLA levels from the batched k-lists
    (csrc/randla_sampler.hip): for every point of the concatenated levels
    (level i = cat[rs[i]:rs[i+1]]), the position within level i+1 of its
    nearest point among the first nxt[i] points of its level —
    knn_search(level i+1, level i, 1) - srs[i] without a second search.
    nb_all (int32, indices into the concatenation) is rewritten IN PLACE to
    indices relative to each row's own level."""
    total = int(rs[-1])
    up = torch.empty(total, dtype=torch.int64, device=cat.device)
    nbytes = _lib.load().o3dml_randla_up_workspace_size(total)
    ws = scratch("up", nbytes) if scratch else torch.empty(nbytes, dtype=torch.uint8, device=cat.device)
    rs, nxt, srs = (np.ascontiguousarray(a, np.int64) for a in (rs, nxt, srs))
    _lib.call("o3dml_randla_up_from_knn", ptr(nb_all), nb_all.shape[1], ptr(cat), len(nxt), rs.ctypes.data,
              nxt.ctypes.data, srs.ctypes.data, ptr(up), ptr(ws), ws.numel(), stream_handle(cat.device))
    return up


def _last_occurrence(idxs, n):
    """Mask of the entries of idxs that are the LAST occurrence of their value:
    numpy's ``a[idxs] += v`` / ``a[idxs] = f(a[idxs])`` (the reference's
    semseg_spatially_regular.py:104 and randlanet.py:462) keep the value of the
    last duplicate — selected here deterministically instead of a racing
    scatter."""
    pos = torch.arange(idxs.shape[0], device=idxs.device)
    last = torch.full((n,), -1, dtype=torch.int64, device=idxs.device)  # idxs < n
    last.scatter_reduce_(0, idxs, pos, reduce="amax")
    return last[idxs] == pos


_CAP_STEP = 16384  # cloud capacity granularity of a patch-step state (and graph)
_FAR = 1.0e9       # padding points: never within a patch of a real point


class _PatchStep:
    """One whole patch of the spatially-regular sampler as a fixed sequence of
    launches over preallocated buffers — crop kNN (k = num_points), keyed
    shuffle (device seed state), possibility update + recentring, the
    per-level k-lists (one batched search), up-sampling ids, the network,
    the test_probs EMA and the next centre (min possibility into pinned
    memory) — with no host synchronisation and no host value that changes
    between patches, so it is captured once as a HIP graph and replayed per
    patch (SemSegInference.run).  The cloud lives in a buffer of ``cap``
    points (sub-sampled cloud + far padding with possibility +inf: never a
    centre, never in a crop), so clouds of similar size reuse the graph.

    The crop is the SET of the num_points nearest points in index order
    (o3dml_knn_select: radix selection, no sort — it is shuffled next).

    replay (tests): the shuffle takes a positional permutation from the
    device buffer ``perm`` (idxs = crop[perm], refreshed by the host before
    each replay) instead of the keyed bijection, so a recorded reference run
    can be replayed through this exact (captured) path."""

    def __init__(self, inf, cap, replay=False):
        model, dev = inf.model, inf.device
        cfg = model.cfg
        lib = _lib.load()
        self.inf, self.cap, self.dev = inf, cap, dev
        k, n_pts = cfg["num_neighbors"], cfg["num_points"]
        self.n_pts = n_pts
        self.sub = torch.empty((cap, 3), dtype=torch.float32, device=dev)
        self.poss = torch.empty(cap, dtype=torch.float64, device=dev)
        self.probs = torch.zeros((cap, cfg["num_classes"]), dtype=inf.probs_dtype, device=dev)
        self.seeds = torch.zeros(2, dtype=torch.int64, device=dev)  # u64 base, counter
        self.arg = torch.empty(1, dtype=torch.int64, device=dev)
        self.center = torch.empty(3, dtype=torch.float32, device=dev)
        self.host_min = torch.empty(1, dtype=torch.float64, pin_memory=True)
        self.min_ws = torch.empty(max(lib.o3dml_randla_possibility_min_workspace_size(), 1), dtype=torch.uint8,
                                  device=dev)
        # crop: one query (the centre) against the padded cloud
        self.crop_ws = torch.empty(max(lib.o3dml_knn_select_workspace_size(cap), 1), dtype=torch.uint8, device=dev)
        self.crop = torch.empty(n_pts, dtype=torch.int64, device=dev)
        self.idxs = torch.empty(n_pts, dtype=torch.int64, device=dev)
        self.pc = torch.empty((n_pts, 3), dtype=torch.float32, device=dev)
        self.patch_ws = torch.empty(max(lib.o3dml_randla_patch_workspace_size(n_pts), 1), dtype=torch.uint8,
                                    device=dev)
        # levels: prefixes of the shuffled patch, one batched self-kNN
        L = cfg["num_layers"]
        sizes = [n_pts]
        for i in range(L):
            sizes.append(sizes[-1] // cfg["sub_sampling_ratio"][i])
        self.sizes = sizes
        self.rs = np.concatenate([[0], np.cumsum(sizes[:L])]).astype(np.int64)
        self.srs = np.concatenate([[0], np.cumsum(sizes[1:])]).astype(np.int64)
        self.nxt = np.asarray(sizes[1:], np.int64)
        total = int(self.rs[-1])
        self.rs_d = torch.from_numpy(self.rs).to(dev)
        self.cat = torch.empty((total, 3), dtype=torch.float32, device=dev)
        self.k = k
        self.knn_rs = torch.empty(total + 1, dtype=torch.int64, device=dev)
        self.knn_ws = torch.empty(max(lib.o3dml_knn_search_workspace_size(total, total, k, L), 1),
                                  dtype=torch.uint8, device=dev)
        self.nb = torch.empty((total, k), dtype=torch.int32, device=dev)
        self.up = torch.empty(total, dtype=torch.int64, device=dev)
        self.up_ws = torch.empty(max(lib.o3dml_randla_up_workspace_size(total), 1), dtype=torch.uint8, device=dev)
        self.plan = (sizes, self.rs, self.srs)
        self.perm = torch.empty(n_pts, dtype=torch.int64, device=dev) if replay else None
        self.graph = None

    def begin(self, sub, poss0, base_seed):
        """Load a frame: the sub-sampled cloud, its initial possibilities, a
        fresh shuffle key; the first centre."""
        n = sub.shape[0]
        self.sub[:n].copy_(sub)
        self.sub[n:].fill_(_FAR)
        self.poss[:n].copy_(poss0)
        self.poss[n:].fill_(float("inf"))
        self.probs.zero_()
        self.seeds.copy_(torch.tensor([base_seed, 0], dtype=torch.int64))
        self._next_centre(stream_handle(self.dev))

    def _next_centre(self, st):
        _lib.call("o3dml_randla_possibility_min", ptr(self.poss), self.cap, ptr(self.sub), ptr(self.arg),
                  ptr(self.center), self.host_min.data_ptr(), ptr(self.min_ws), self.min_ws.numel(), st)

    def step(self):
        """The launches of one patch (graph-capturable)."""
        inf, st, n_pts = self.inf, stream_handle(self.dev), self.n_pts
        k, L = self.k, len(self.nxt)
        # crop: the SET of the num_points nearest sub-points of the centre, in
        # index order (radix selection, nns_topk.hip; shuffled next)
        l2 = metric_code("L2")
        _lib.call("o3dml_knn_select", ptr(self.sub), self.cap, ptr(self.center), n_pts, l2, ptr(self.crop),
                  ptr(self.crop_ws), self.crop_ws.numel(), st)
        # the shuffle (random.shuffle, semseg_spatially_regular.py:100): keyed
        # bijection, or (replay) the injected positional permutation
        if self.perm is not None:
            torch.index_select(self.crop, 0, self.perm, out=self.idxs)
        else:
            _lib.call("o3dml_random_permute_dev", ptr(self.crop), n_pts, ptr(self.seeds), ptr(self.idxs), st)
        # pc = sub[idxs], possibilities += delta, x / y recentred
        _lib.call("o3dml_randla_patch_update", ptr(self.sub), ptr(self.idxs), n_pts, ptr(self.center), None,
                  ptr(self.poss), ptr(self.pc), ptr(self.patch_ws), self.patch_ws.numel(), st)
        torch.cat([self.pc[:self.sizes[i]] for i in range(L)], out=self.cat)
        total = self.cat.shape[0]
        _lib.call("o3dml_knn_search_count", ptr(self.cat), total, ptr(self.cat), total, k, L, ptr(self.rs_d),
                  ptr(self.rs_d), self.rs.ctypes.data, self.rs.ctypes.data, l2, 0, 1, ptr(self.knn_rs),
                  ptr(self.knn_ws), self.knn_ws.numel(), st)
        _lib.call("o3dml_knn_search_fill", ptr(self.cat), total, ptr(self.cat), total, k, L, ptr(self.rs_d),
                  self.rs.ctypes.data, self.rs.ctypes.data, l2, 0, ptr(self.knn_rs), 32, ptr(self.nb), None,
                  ptr(self.knn_ws), self.knn_ws.numel(), st)
        _lib.call("o3dml_randla_up_from_knn", ptr(self.nb), k, ptr(self.cat), L, self.rs.ctypes.data,
                  self.nxt.ctypes.data, self.srs.ctypes.data, ptr(self.up), ptr(self.up_ws), self.up_ws.numel(), st)
        probs = inf._patch_probs(self.pc, self.nb, self.up, self.plan)
        inf.update_probs(self.probs, self.idxs, probs)
        self._next_centre(st)

    def run_step(self, use_graph):
        if not use_graph:
            self.step()
            return
        if self.graph is None:
            # warm-up outside the capture (allocator, lazy library state), on
            # a state copy: the warm-up must not move this frame's state
            saved = (self.poss.clone(), self.probs.clone(), self.seeds.clone(), self.center.clone(),
                     self.arg.clone())
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.step()
            torch.cuda.current_stream(self.dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.step()
            for t, v in zip((self.poss, self.probs, self.seeds, self.center, self.arg), saved):
                t.copy_(v)
            self.graph = g
        self.graph.replay()


class SemSegInference:
    """GPU ``run_inference`` for RandLA-Net with the spatially-regular patch
    sampler.  ``run(points)`` -> (predicted labels [N] int64, probabilities
    [N, C]), both on the GPU; ``stats`` records patches per frame.

    Arithmetic as in the reference (semseg_spatially_regular.py:79-109,
    randlanet.py:441-465, semantic_segmentation.py:264-299): possibilities in
    float64 with float32 ``delta = (1 - d / d_max)^2``, centre = first argmin;
    the per-point probabilities stored in float16 as the reference's
    ``test_probs`` (update ``f16(f16(0.95) * p16 + f32(0.05) * probs)``;
    ``probs_dtype=torch.float32`` keeps them in f32); duplicate patch indices
    (clouds smaller than a patch) take the last duplicate's value, as numpy's
    fancy-index assignment does.  ``run(points, patch_hook=f,
    init_possibility=p0)`` replays a recorded patch order: f(patch_number,
    centre_id) returns the patch's (already shuffled) indices in place of the
    GPU kNN crop + shuffle (tests/test_gpu_pipeline.py).  ``run(points,
    perm_hook=g, init_possibility=p0)`` replays one through the timed path
    itself (the captured whole-patch step): g(patch_number, centre_id)
    returns the positional permutation of the GPU crop (the crop set in
    index order) that gives the recorded patch; the centres and each patch's
    indices land in ``stats``."""

    def __init__(self, model, device=None, seed=0, test_smooth=0.95, use_graph=None, probs_dtype=torch.float16):
        self.model = model
        if use_graph is None:
            use_graph = os.environ.get("O3DML_RANDLA_GRAPH", "1") != "0"
        self.use_graph = use_graph
        self.device = device or next(model.parameters()).device
        self.test_smooth = test_smooth
        self.probs_dtype = probs_dtype
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.rng = np.random.default_rng(seed)  # patch-shuffle keys (host side: no device round trip)
        self.stats = {}

    def preprocess(self, points):
        """Grid subsampling + 1-NN projection of every raw point (randlanet.py:115-152), once."""
        cfg = self.model.cfg
        sub, _, _, _ = ops.grid_subsample(points, [points.shape[0]], cfg["grid_size"])
        proj = ops.knn_search(sub, points, 1).neighbors_index.long()
        return sub, proj

    def transform(self, sub, possibility, center, idxs=None):
        """Patch crop + possibility update + per-layer kNN (randlanet.py:156-239,
        semseg_spatially_regular.py:82-109).  center: the device centre point
        [3] (o3dml_randla_possibility_min); idxs: a replayed patch (shuffled
        indices) instead of the crop."""
        cfg = self.model.cfg
        n_pts = cfg["num_points"]
        dev = self.device
        if idxs is not None:
            idxs = idxs.to(dev).long().contiguous()
        else:
            if sub.shape[0] < n_pts:
                extra = torch.randint(0, sub.shape[0], (n_pts - sub.shape[0],), generator=self.gen, device=dev)
                crop = torch.cat([torch.arange(sub.shape[0], device=dev), extra])
            else:
                crop = ops.knn_search(sub, center.view(1, 3), n_pts, index_dtype=torch.int64).neighbors_index
            # the shuffle (random.shuffle, semseg_spatially_regular.py:100): a
            # keyed random bijection, one launch (o3dml_random_permute)
            idxs = torch.empty_like(crop)
            _lib.call("o3dml_random_permute", ptr(crop), crop.shape[0], int(self.rng.integers(0, 2**63)),
                      ptr(idxs), stream_handle(dev))
        # duplicates (a cloud smaller than a patch): the last one's value, as
        # numpy's possibilities[idxs] += delta
        keep = _last_occurrence(idxs, sub.shape[0]).to(torch.uint8) if sub.shape[0] < idxs.shape[0] else None
        # pc = sub[idxs], delta = (1 - d / d_max)^2 into the float64
        # possibilities, x / y recentred (csrc/randla_sampler.hip)
        pc = torch.empty((idxs.shape[0], 3), dtype=torch.float32, device=dev)
        ws = self._ws("patch", _lib.load().o3dml_randla_patch_workspace_size(idxs.shape[0]))
        _lib.call("o3dml_randla_patch_update", ptr(sub), ptr(idxs), idxs.shape[0], ptr(center), ptr(keep),
                  ptr(possibility), ptr(pc), ptr(ws), ws.numel(), stream_handle(dev))
        # all levels are prefixes of the shuffled patch: one batched self-kNN
        # (k=16) covers the 4 layers; the up-sampling indices come from its
        # sorted lists (o3dml_randla_up_from_knn == knn(level i+1, level i, 1))
        L = cfg["num_layers"]
        sizes = [pc.shape[0]]
        for i in range(L):
            sizes.append(sizes[-1] // cfg["sub_sampling_ratio"][i])
        levels = [pc[:sizes[i]] for i in range(L)]
        k = cfg["num_neighbors"]
        cat = torch.cat(levels).contiguous()
        rs = np.concatenate([[0], np.cumsum(sizes[:L])]).astype(np.int64)
        nb_all = ops.knn_search(cat, cat, k, rs, rs).neighbors_index.view(-1, k)
        srs = np.concatenate([[0], np.cumsum(sizes[1:])]).astype(np.int64)
        up_all = up_from_knn(nb_all, cat, rs, np.asarray(sizes[1:], np.int64), srs, self._ws)
        return pc, idxs, nb_all, up_all, (sizes, rs, srs)

    def _ws(self, name, nbytes):
        """Per-pipeline device scratch (grown on demand, reused across patches)."""
        buf = self.__dict__.setdefault("_scratch", {}).get(name)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.device)
            self._scratch[name] = buf
        return buf

    def update_probs(self, test_probs, idxs, probs):
        """test_probs[idxs] = smooth * test_probs[idxs] + (1 - smooth) * probs
        (randlanet.py:441-465) with the reference's dtypes: a float16 store
        multiplies in float16 (numpy casts the Python scalar to the array's
        dtype), the new term is float32, the sum float32 rounded to the store;
        duplicate indices keep the last one (numpy semantics)."""
        keep = None
        if test_probs.shape[0] < idxs.shape[0]:  # a patch larger than the cloud repeats points
            keep = _last_occurrence(idxs, test_probs.shape[0]).to(torch.uint8)
        _lib.call("o3dml_randla_update_probs", ptr(probs.float().contiguous()), ptr(idxs), ptr(keep), idxs.shape[0],
                  test_probs.shape[1], float(self.test_smooth), int(test_probs.dtype == torch.float16),
                  ptr(test_probs), stream_handle(test_probs.device))

    def _levels(self, pc, nb_all, up_all, plan):
        """Per-layer (coords, nbrs, subs, ups) views of the batched kNN results
        (already level-relative: up_from_knn); no kernels."""
        sizes, rs, srs = plan
        coords, nbrs, subs, ups = [], [], [], []
        for i in range(self.model.cfg["num_layers"]):
            nb = nb_all[rs[i]:rs[i + 1]]
            coords.append(pc[:sizes[i]])
            nbrs.append(nb)
            subs.append(nb[:sizes[i + 1]])
            ups.append(up_all[rs[i]:rs[i + 1]])
        return coords, nbrs, subs, ups

    def _patch_probs(self, pc, nb_all, up_all, plan):
        coords, nbrs, subs, ups = self._levels(pc, nb_all, up_all, plan)
        return torch.softmax(self.model.forward_points(pc, coords, nbrs, subs, ups), -1)

    def _graph_probs(self, pc, nb_all, up_all, plan):
        """The network part of a patch (per-layer views, forward, softmax: ~100
        launches) replayed as one HIP graph: every full-size patch has the same
        shapes, so the graph is captured once per (model, patch plan) and its
        static inputs are refreshed with three device copies.  The graph lives on
        the model (one per patch plan and device), so later frames reuse it."""
        key = (str(self.device), tuple(plan[0]))
        g = self.model.__dict__.get("_o3dml_patch_graph")
        if g is None or g[0] != key:
            st = {"pc": pc.clone(), "nb": nb_all.clone(), "up": up_all.clone()}
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                for _ in range(2):  # warm-up outside the capture (caches, allocator)
                    self._patch_probs(st["pc"], st["nb"], st["up"], plan)
            torch.cuda.current_stream(self.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._patch_probs(st["pc"], st["nb"], st["up"], plan)
            g = self.model.__dict__["_o3dml_patch_graph"] = (key, graph, st, out)
        _, graph, st, out = g
        st["pc"].copy_(pc)
        st["nb"].copy_(nb_all)
        st["up"].copy_(up_all)
        graph.replay()
        return out

    _MAX_STEPS = 4  # patch-step states (and graphs) kept per model

    def _patch_step(self, n_sub, replay=False):
        """The patch-step state (and its graph) for a cloud of n_sub points,
        kept on the model per (device, capacity, dtype, smooth, replay): up to
        _MAX_STEPS of them, so scans whose sub-clouds fall into a few
        capacity classes do not re-capture the graph when they alternate."""
        cap = -(-n_sub // _CAP_STEP) * _CAP_STEP
        key = (str(self.device), cap, self.probs_dtype, self.test_smooth, bool(replay))
        steps = self.model.__dict__.setdefault("_o3dml_patch_step", {})
        step = steps.pop(key, None)
        if step is None:
            step = _PatchStep(self, cap, replay)
            while len(steps) >= self._MAX_STEPS:
                steps.pop(next(iter(steps)))  # least recently used first
        steps[key] = step  # most recently used last
        step.inf = self
        return step

    @torch.no_grad()
    def run(self, points, patch_hook=None, init_possibility=None, perm_hook=None):
        self.model.eval()
        self.model._sync_folded()
        points = points.to(self.device).float().contiguous()
        C = self.model.cfg["num_classes"]
        sub, proj = self.preprocess(points)
        n_sub = sub.shape[0]
        if init_possibility is not None:
            possibility = torch.as_tensor(init_possibility, dtype=torch.float64).to(self.device).clone()
        else:
            possibility = torch.rand(n_sub, generator=self.gen, device=self.device, dtype=torch.float64) * 1e-3
        if patch_hook is None and n_sub >= self.model.cfg["num_points"]:
            # the whole patch as one replayed graph (or the same launches eagerly)
            step = self._patch_step(n_sub, replay=perm_hook is not None)
            step.begin(sub, possibility, int(self.rng.integers(0, 2**63)))
            patches, centers, patch_idxs = 0, [], []
            ready = torch.cuda.Event()
            while True:
                ready.record(torch.cuda.current_stream(self.device))
                ready.synchronize()
                if float(step.host_min[0]) > 0.5:
                    break
                if perm_hook is not None:  # replay (tests): the recorded shuffle, the centre on the host
                    cid = int(step.arg.item())
                    centers.append(cid)
                    step.perm.copy_(torch.as_tensor(np.asarray(perm_hook(patches, cid), np.int64)))
                step.run_step(self.use_graph)
                if perm_hook is not None:
                    patch_idxs.append(step.idxs.clone())
                patches += 1
            self.stats = {"patches": patches, "sub_points": n_sub, "centers": centers}
            if perm_hook is not None:
                self.stats["patch_idxs"] = patch_idxs
            probs = step.probs[:n_sub][proj]
            return probs.argmax(1), probs
        test_probs = torch.zeros((n_sub, C), dtype=self.probs_dtype, device=self.device)
        patches, centers = 0, []
        arg = torch.empty(1, dtype=torch.int64, device=self.device)
        center = torch.empty(3, dtype=torch.float32, device=self.device)
        host_min = torch.empty(1, dtype=torch.float64, pin_memory=True)
        mws = self._ws("min", _lib.load().o3dml_randla_possibility_min_workspace_size())
        st = stream_handle(self.device)
        ready = torch.cuda.Event()
        while True:
            # min + first argmin of the possibilities, the centre point; the
            # minimum straight into pinned memory: the one host read per patch
            _lib.call("o3dml_randla_possibility_min", ptr(possibility), n_sub, ptr(sub), ptr(arg), ptr(center),
                      host_min.data_ptr(), ptr(mws), mws.numel(), st)
            ready.record(torch.cuda.current_stream(self.device))
            ready.synchronize()
            if float(host_min[0]) > 0.5:
                break
            idxs = None
            if patch_hook is not None:
                cid = int(arg.item())
                centers.append(cid)
                idxs = patch_hook(patches, cid)
            pc, idxs, nb_all, up_all, plan = self.transform(sub, possibility, center, idxs)
            if self.use_graph and n_sub >= self.model.cfg["num_points"]:
                probs = self._graph_probs(pc, nb_all, up_all, plan)
            else:
                probs = self._patch_probs(pc, nb_all, up_all, plan)
            self.update_probs(test_probs, idxs, probs)
            patches += 1
        self.stats = {"patches": patches, "sub_points": n_sub, "centers": centers}
        probs = test_probs[proj]
        return probs.argmax(1), probs
