"""KPFCNN on MI355X: the reference segmentation network and its collate on the
GPU (reference ml3d/torch/models/kpconv.py
KPFCNN :29-291, blocks :1173-1510, pooling :821-858, batch_neighbors
:2002-2034, batch_grid_subsampling :2037-2164, and
ml3d/torch/dataloaders/concat_batcher.py segmentation_inputs :186-283).

* The module tree (``encoder_blocks`` / ``decoder_blocks`` / ``head_mlp`` /
  ``head_softmax`` and every block's sub-module names) is the reference's, so
  reference state_dicts load unchanged and the forward takes the same batch
  object (``points``, ``neighbors``, ``pools``, ``upsamples``, ``lengths``,
  ``features``, ``labels``).
* ``segmentation_inputs`` builds that batch on the GPU: per layer one
  fixed-radius search (HIP, canonical neighbour order) densified by
  ``ragged_to_dense`` with the shadow index, grid subsampling of the randomly
  rotated cloud (HIP) rotated back, and the pool / upsample searches.  The
  reference does this in numpy inside DataLoader workers.
* ``max_pool`` / ``closest_pool`` are HIP kernels with their backward
  (csrc/kpconv.hip ``pool_max_kernel``); KPConv itself is the fused
  neighbourhood aggregation + dense GEMM of ``o3dml_amd.kpconv``.
"""
import threading

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from ._util import index_bits, ptr, stream_handle, to_dev, workspace
from .batchnorm import bn_act, linear_bn_act
from .kpconv import KPConv


# ---------------------------------------------------------------------------
# pooling (kpconv.py:821-858)
# ---------------------------------------------------------------------------
class _PoolMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, inds, nb):
        x = x.contiguous()
        inds = inds.contiguous()
        n, ld = inds.shape
        ns, c = x.shape
        out = torch.empty((n, c), dtype=torch.float32, device=x.device)
        arg = torch.empty((n, c), dtype=torch.int32, device=x.device) if ctx.needs_input_grad[0] else None
        if n and c:
            _lib.call("o3dml_kpconv_pool_max", ptr(x), ns, c, ptr(inds), index_bits(inds.dtype), ld, n, nb, ptr(out),
                      ptr(arg), stream_handle(x.device))
        ctx.save_for_backward(arg, inds)
        ctx.shape = (ns, c, nb)
        return out

    @staticmethod
    def backward(ctx, g):
        arg, inds = ctx.saved_tensors
        ns, c, nb = ctx.shape
        n, ld = inds.shape
        if c and ns and torch.are_deterministic_algorithms_enabled():
            # fixed-order gather over the inverse of inds (no fp32 atomics)
            dx = torch.empty((ns, c), dtype=torch.float32, device=g.device)
            ws = workspace(_lib.load().o3dml_kpconv_inverse_workspace_size(n, nb, ns), g.device)
            _lib.call("o3dml_kpconv_pool_max_backward_det", ptr(g.contiguous()), ptr(arg), ptr(inds),
                      index_bits(inds.dtype), ld, n, nb, c, ns, ptr(dx), ptr(ws), ws.numel(), stream_handle(g.device))
            return dx, None, None
        dx = torch.zeros((ns, c), dtype=torch.float32, device=g.device)
        if n and c:
            _lib.call("o3dml_kpconv_pool_max_backward", ptr(g.contiguous()), ptr(arg), n, c, ns, ptr(dx),
                      stream_handle(g.device))
        return dx, None, None


def _index(inds, dev):
    if inds.device != dev:
        inds = inds.to(dev)
    if inds.dtype not in (torch.int32, torch.int64):
        inds = inds.long()
    return inds


def max_pool(x, inds):
    """[n1, d] features, [n2, max_num] indices (n1 = shadow row of zeros) ->
    [n2, d] max over the row (kpconv.py:840-858)."""
    if x.dim() != 2 or inds.dim() != 2:
        raise RuntimeError("max_pool: x must be [N, D] and inds [M, K]")
    return _PoolMax.apply(x.float(), _index(inds, x.device), inds.shape[1])


def closest_pool(x, inds):
    """Features of each row's first neighbour (n1 = shadow row of zeros)
    (kpconv.py:821-837; assumes column 0 is the closest)."""
    if x.dim() != 2 or inds.dim() != 2:
        raise RuntimeError("closest_pool: x must be [N, D] and inds [M, K]")
    return _PoolMax.apply(x.float(), _index(inds, x.device), 1 if inds.shape[1] else 0)


def global_average(x, batch_lengths):
    """Per-cloud mean (kpconv.py:861-890)."""
    lengths = [int(v) for v in batch_lengths]
    return torch.stack([c.mean(dim=0) for c in torch.split(x, lengths, dim=0)])


# ---------------------------------------------------------------------------
# blocks (kpconv.py:1173-1510) — same module / parameter names
# ---------------------------------------------------------------------------
class BatchNormBlock(nn.Module):
    """BatchNorm1d over the point axis, or a bias when BN is off (kpconv.py:1213-1252).
    BatchNorm1d on [N, C] has the statistics of the reference's [1, C, N] view."""

    def __init__(self, in_dim, use_bn, bn_momentum):
        super().__init__()
        self.bn_momentum = 1 - bn_momentum
        self.use_bn = use_bn
        self.in_dim = in_dim
        if use_bn:
            self.batch_norm = nn.BatchNorm1d(in_dim, momentum=1 - bn_momentum)
        else:
            self.bias = nn.Parameter(torch.zeros(in_dim, dtype=torch.float32))

    def forward(self, x, slope=None):
        """BN (+ LeakyReLU(slope) when slope is not None: the activation the
        enclosing block applies next, fused into the BN launches, csrc/bn.hip)."""
        if self.use_bn:
            return bn_act(x, self.batch_norm, slope)
        x = x + self.bias
        return x if slope is None else F.leaky_relu(x, slope)


class UnaryBlock(nn.Module):
    """Linear (no bias) + BatchNormBlock + LeakyReLU (kpconv.py:1255-1295)."""

    def __init__(self, in_dim, out_dim, use_bn, bn_momentum, no_relu=False, l_relu=0.1):
        super().__init__()
        self.bn_momentum = bn_momentum
        self.use_bn = use_bn
        self.no_relu = no_relu
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.mlp = nn.Linear(in_dim, out_dim, bias=False)
        self.batch_norm = BatchNormBlock(out_dim, use_bn, bn_momentum)
        if not no_relu:
            self.leaky_relu = nn.LeakyReLU(l_relu)

    def forward(self, x, batch=None):
        slope = None if self.no_relu else self.leaky_relu.negative_slope
        if self.use_bn:  # Linear + BN (+ LeakyReLU) as one autograd node (batchnorm.linear_bn_act)
            return linear_bn_act(x, self.mlp.weight, self.batch_norm.batch_norm, slope)
        return self.batch_norm(self.mlp(x), slope)


def _conv_inputs(block_name, layer_ind, batch):
    if "strided" in block_name:
        return batch.points[layer_ind + 1], batch.points[layer_ind], batch.pools[layer_ind]
    return batch.points[layer_ind], batch.points[layer_ind], batch.neighbors[layer_ind]


def _kpconv(config, in_dim, out_dim, radius, block_name):
    extent = radius * config.KP_extent / config.conv_radius
    return KPConv(config.num_kernel_points, config.in_points_dim, in_dim, out_dim, extent, radius,
                  fixed_kernel_points=config.fixed_kernel_points, KP_influence=config.KP_influence,
                  aggregation_mode=config.aggregation_mode, deformable="deform" in block_name,
                  modulated=config.modulated)


class SimpleBlock(nn.Module):
    """KPConv + BN + LeakyReLU, out_dim // 2 channels (kpconv.py:1298-1357)."""

    def __init__(self, block_name, in_dim, out_dim, radius, layer_ind, config):
        super().__init__()
        self.bn_momentum = config.batch_norm_momentum
        self.use_bn = config.use_batch_norm
        self.layer_ind = layer_ind
        self.block_name = block_name
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.KPConv = _kpconv(config, in_dim, out_dim // 2, radius, block_name)
        self.batch_norm = BatchNormBlock(out_dim // 2, self.use_bn, self.bn_momentum)
        self.leaky_relu = nn.LeakyReLU(config.get("l_relu", 0.1))

    def forward(self, x, batch):
        q, s, nb = _conv_inputs(self.block_name, self.layer_ind, batch)
        return self.batch_norm(self.KPConv(q, s, nb, x), self.leaky_relu.negative_slope)


class ResnetBottleneckBlock(nn.Module):
    """unary1 -> KPConv -> BN/LReLU -> unary2, + (max-pooled) shortcut
    (kpconv.py:1360-1464)."""

    def __init__(self, block_name, in_dim, out_dim, radius, layer_ind, config):
        super().__init__()
        self.bn_momentum = config.batch_norm_momentum
        self.use_bn = config.use_batch_norm
        self.block_name = block_name
        self.layer_ind = layer_ind
        self.in_dim = in_dim
        self.out_dim = out_dim
        l_relu = config.get("l_relu", 0.1)
        if in_dim != out_dim // 4:
            self.unary1 = UnaryBlock(in_dim, out_dim // 4, self.use_bn, self.bn_momentum, l_relu=l_relu)
        else:
            self.unary1 = nn.Identity()
        self.KPConv = _kpconv(config, out_dim // 4, out_dim // 4, radius, block_name)
        self.batch_norm_conv = BatchNormBlock(out_dim // 4, self.use_bn, self.bn_momentum)
        self.unary2 = UnaryBlock(out_dim // 4, out_dim, self.use_bn, self.bn_momentum, no_relu=True, l_relu=l_relu)
        if in_dim != out_dim:
            self.unary_shortcut = UnaryBlock(in_dim, out_dim, self.use_bn, self.bn_momentum, no_relu=True,
                                             l_relu=l_relu)
        else:
            self.unary_shortcut = nn.Identity()
        self.leaky_relu = nn.LeakyReLU(l_relu)

    def forward(self, features, batch):
        q, s, nb = _conv_inputs(self.block_name, self.layer_ind, batch)
        x = self.unary1(features)
        x = self.batch_norm_conv(self.KPConv(q, s, nb, x), self.leaky_relu.negative_slope)
        x = self.unary2(x)
        shortcut = max_pool(features, nb) if "strided" in self.block_name else features
        return self.leaky_relu(x + self.unary_shortcut(shortcut))


class GlobalAverageBlock(nn.Module):
    def forward(self, x, batch):
        return global_average(x, batch.lengths[-1])


class NearestUpsampleBlock(nn.Module):
    def __init__(self, layer_ind):
        super().__init__()
        self.layer_ind = layer_ind

    def forward(self, x, batch):
        return closest_pool(x, batch.upsamples[self.layer_ind - 1])


class MaxPoolBlock(nn.Module):
    def __init__(self, layer_ind):
        super().__init__()
        self.layer_ind = layer_ind

    def forward(self, x, batch):
        return max_pool(x, batch.pools[self.layer_ind + 1])


def block_decider(block_name, radius, in_dim, out_dim, layer_ind, config):
    """kpconv.py:1173-1210."""
    if block_name == "unary":
        return UnaryBlock(in_dim, out_dim, config.use_batch_norm, config.batch_norm_momentum,
                          l_relu=config.get("l_relu", 0.1))
    if block_name.startswith("simple"):
        return SimpleBlock(block_name, in_dim, out_dim, radius, layer_ind, config)
    if block_name.startswith("resnetb"):
        return ResnetBottleneckBlock(block_name, in_dim, out_dim, radius, layer_ind, config)
    if block_name in ("max_pool", "max_pool_wide"):
        return MaxPoolBlock(layer_ind)
    if block_name == "global_average":
        return GlobalAverageBlock()
    if block_name == "nearest_upsample":
        return NearestUpsampleBlock(layer_ind)
    raise ValueError("Unknown block name in the architecture definition : " + block_name)


class Config(dict):
    """Attribute-access dict (the reference's addict config)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)


DEFAULTS = dict(
    name="KPFCNN", lbl_values=list(range(20)), num_classes=19, ignored_label_inds=[0],
    architecture=["simple", "resnetb", "resnetb_strided", "resnetb", "resnetb", "resnetb_strided", "resnetb",
                  "resnetb", "resnetb_strided", "resnetb", "resnetb", "resnetb_strided", "resnetb",
                  "nearest_upsample", "unary", "nearest_upsample", "unary", "nearest_upsample", "unary",
                  "nearest_upsample", "unary"],
    in_radius=4.0, max_in_points=100000, batch_num=8, batch_limit=30000, val_batch_num=8, num_kernel_points=15,
    first_subsampling_dl=0.06, conv_radius=2.5, deform_radius=6.0, KP_extent=1.2, KP_influence="linear",
    aggregation_mode="sum", first_features_dim=128, in_features_dim=2, modulated=False, use_batch_norm=True,
    batch_norm_momentum=0.02, deform_fitting_mode="point2point", deform_fitting_power=1.0, repulse_extent=1.2,
    in_points_dim=3, fixed_kernel_points="center", num_layers=5, l_relu=0.1, reduce_fc=False)

# sparseconvunet-style preset of the reference's ml3d/configs/kpconv_s3dis.yml (model section)
S3DIS = dict(lbl_values=list(range(13)), num_classes=13, ignored_label_inds=[], first_subsampling_dl=0.04,
             in_features_dim=5, in_radius=1.5, batch_limit=20000, max_in_points=20000, batch_norm_momentum=0.98)


class KPFCNN(nn.Module):
    """Reference-compatible KPFCNN (kpconv.py:29-291): same constructor
    arguments, same module tree, same forward over a KPConv batch."""

    def __init__(self, **kwargs):
        super().__init__()
        cfg = Config(DEFAULTS)
        cfg.update(kwargs)
        self.cfg = cfg
        layer = 0
        r = cfg.first_subsampling_dl * cfg.conv_radius
        in_dim = cfg.in_features_dim
        out_dim = cfg.first_features_dim
        self.K = cfg.num_kernel_points
        self.C = len(cfg.lbl_values) - len(cfg.ignored_label_inds)

        self.encoder_blocks = nn.ModuleList()
        self.encoder_skip_dims = []
        self.encoder_skips = []
        self.neighborhood_limits = []
        for block_i, block in enumerate(cfg.architecture):
            if "equivariant" in block and out_dim % 3 != 0:
                raise ValueError("Equivariant block but features dimension is not a factor of 3")
            if any(t in block for t in ("pool", "strided", "upsample", "global")):
                self.encoder_skips.append(block_i)
                self.encoder_skip_dims.append(in_dim)
            if "upsample" in block:
                break
            self.encoder_blocks.append(block_decider(block, r, in_dim, out_dim, layer, cfg))
            in_dim = out_dim // 2 if "simple" in block else out_dim
            if "pool" in block or "strided" in block:
                layer += 1
                r *= 2
                out_dim *= 2

        self.decoder_blocks = nn.ModuleList()
        self.decoder_concats = []
        start_i = next((i for i, b in enumerate(cfg.architecture) if "upsample" in b), 0)
        for block_i, block in enumerate(cfg.architecture[start_i:]):
            if block_i > 0 and "upsample" in cfg.architecture[start_i + block_i - 1]:
                in_dim += self.encoder_skip_dims[layer]
                self.decoder_concats.append(block_i)
            self.decoder_blocks.append(block_decider(block, r, in_dim, out_dim, layer, cfg))
            in_dim = out_dim
            if block_i == 0 and cfg.reduce_fc:
                out_dim = out_dim // 2
            if "upsample" in block:
                layer -= 1
                r *= 0.5
                out_dim = out_dim // 2

        l_relu = cfg.get("l_relu", 0.1)
        if cfg.reduce_fc:
            self.head_mlp = UnaryBlock(out_dim, cfg.first_features_dim // 2, True, cfg.batch_norm_momentum,
                                       l_relu=l_relu)
            self.head_softmax = UnaryBlock(cfg.first_features_dim // 2, self.C, False, 1, no_relu=True,
                                           l_relu=l_relu)
        else:
            self.head_mlp = UnaryBlock(out_dim, cfg.first_features_dim, False, 0, l_relu=l_relu)
            self.head_softmax = UnaryBlock(cfg.first_features_dim, self.C, False, 0, l_relu=l_relu)
        self.valid_labels = np.sort([c for c in cfg.lbl_values if c not in cfg.ignored_label_inds])
        self.deform_fitting_mode = cfg.deform_fitting_mode
        self.deform_fitting_power = cfg.deform_fitting_power
        self.repulse_extent = cfg.repulse_extent

    def forward(self, batch):
        x = batch.features.clone().detach()
        skip_x = []
        for block_i, block_op in enumerate(self.encoder_blocks):
            if block_i in self.encoder_skips:
                skip_x.append(x)
            x = block_op(x, batch)
        for block_i, block_op in enumerate(self.decoder_blocks):
            if block_i in self.decoder_concats:
                x = torch.cat([x, skip_x.pop()], dim=1)
            x = block_op(x, batch)
        x = self.head_mlp(x, batch)
        return self.head_softmax(x, batch)

    def get_loss(self, logits, labels, class_weights=None):
        """Cross entropy over the valid labels + the point-to-point fitting
        regulariser of the deformable KPConvs (kpconv.py:315-351; zero for the
        rigid architectures).  The parts are kept as output_loss / reg_loss."""
        self.output_loss = self._ce(logits, labels, class_weights)
        if self.deform_fitting_mode != "point2point":
            raise ValueError("Unknown fitting mode: " + str(self.deform_fitting_mode))
        self.reg_loss = p2p_fitting_regularizer(self)
        return self.output_loss + self.reg_loss

    def _ce(self, logits, labels, class_weights=None):
        labels = labels.to(logits.device).long()
        valid = torch.ones_like(labels, dtype=torch.bool)
        for ign in self.cfg.ignored_label_inds:
            valid &= labels != ign
        lut = torch.full((max(self.cfg.lbl_values) + 1,), -1, dtype=torch.long, device=logits.device)
        lut[torch.as_tensor(self.valid_labels, device=logits.device)] = torch.arange(len(self.valid_labels),
                                                                                     device=logits.device)
        w = None if class_weights is None else torch.as_tensor(class_weights, dtype=torch.float32,
                                                               device=logits.device)
        return F.cross_entropy(logits[valid], lut[labels[valid]], weight=w)


def p2p_fitting_regularizer(net):
    """kpconv.py:2167-2209: for every deformable KPConv, the L1 mean of the
    normalised squared distance from each deformed kernel point to its nearest
    input point (fitting) and a repulsion between the normalised kernel points
    of one query (other points detached); deform_fitting_power * (2 * fitting
    + repulsive).  min_d2 / deformed_KP come from the last forward
    (kpconv.min_d2: the distances differentiate into the kernel points)."""
    fitting = 0
    repulsive = 0
    l1 = torch.nn.functional.l1_loss
    for m in net.modules():
        if isinstance(m, KPConv) and m.deformable:
            kp_min_d2 = m.min_d2 / (m.KP_extent ** 2)
            fitting = fitting + l1(kp_min_d2, torch.zeros_like(kp_min_d2))
            locs = m.deformed_KP / m.KP_extent
            for i in range(net.K):
                other = torch.cat([locs[:, :i, :], locs[:, i + 1:, :]], dim=1).detach()
                dist = torch.sqrt(torch.sum((other - locs[:, i:i + 1, :]) ** 2, dim=2))
                rep = torch.sum(torch.clamp_max(dist - net.repulse_extent, max=0.0) ** 2, dim=1)
                repulsive = repulsive + l1(rep, torch.zeros_like(rep)) / net.K
    return net.deform_fitting_power * (2 * fitting + repulsive)


# ---------------------------------------------------------------------------
# GPU collate (concat_batcher.py:186-283, kpconv.py:2002-2164)
# ---------------------------------------------------------------------------
class KPConvBatch:
    """The attributes KPFCNN.forward reads (concat_batcher.py KPConvBatch)."""

    def __init__(self, points, neighbors, pools, upsamples, lengths, features, labels):
        self.points = points
        self.neighbors = neighbors
        self.pools = pools
        self.upsamples = upsamples
        self.lengths = lengths
        self.features = features
        self.labels = labels


def random_rotations(B, rng=np.random):
    """Random 3D rotations as batch_grid_subsampling draws them
    (kpconv.py:2063-2080): axis from two polar angles, angle U[0, 2pi),
    Rodrigues' matrix, float32 [B, 3, 3]; applied as p @ R."""
    theta = rng.rand(B) * 2 * np.pi
    phi = (rng.rand(B) - 0.5) * np.pi
    u = np.stack([np.cos(theta) * np.cos(phi), np.sin(theta) * np.cos(phi), np.sin(phi)], axis=1)
    alpha = rng.rand(B) * 2 * np.pi
    c, s = np.cos(alpha)[:, None, None], np.sin(alpha)[:, None, None]
    cross = np.zeros((B, 3, 3))
    cross[:, 0, 1], cross[:, 0, 2], cross[:, 1, 2] = -u[:, 2], u[:, 1], -u[:, 0]
    cross -= cross.transpose(0, 2, 1)
    R = c * np.eye(3)[None] + (1 - c) * u[:, :, None] * u[:, None, :] + s * cross
    return R.astype(np.float32)


def _rotate(points, splits, R, transpose=False):
    """p' = p @ R[b] per batch element in fp32 with the reference's rounding
    ((p0 R0j + p1 R1j) + p2 R2j, each product rounded; kpconv.py:2087-2090):
    one HIP launch (o3dml_rotate_batched), the rotations through a pinned
    non-blocking upload."""
    dev = points.device
    pts = points.contiguous()
    out = torch.empty_like(pts)
    B = len(splits) - 1
    _lib.call("o3dml_rotate_batched", ptr(pts), pts.shape[0], B, ptr(to_dev(np.asarray(splits, np.int64), dev)),
              ptr(to_dev(np.ascontiguousarray(R, np.float32), dev)), int(bool(transpose)), ptr(out),
              stream_handle(dev))
    return out


def batch_grid_subsampling(points, lengths, sampleDl, rotations=None, random_grid_orient=True):
    """Grid subsampling per batch element in a random orientation, rotated
    back (kpconv.py:2037-2164).  points GPU f32 [N,3], lengths host ints ->
    (sub points [S,3], sub lengths np.int64 [B])."""
    lengths = np.asarray(lengths, np.int64)
    splits = np.zeros(len(lengths) + 1, np.int64)
    splits[1:] = np.cumsum(lengths)
    R = None
    if random_grid_orient:
        R = random_rotations(len(lengths)) if rotations is None else np.asarray(rotations, np.float32)
        points = _rotate(points, splits, R)
    out = ops.grid_subsample(points, lengths, sampleDl)
    s_len = out.lengths.cpu().numpy()
    s_pts = out.points
    if random_grid_orient:
        s_splits = np.zeros(len(s_len) + 1, np.int64)
        s_splits[1:] = np.cumsum(s_len)
        s_pts = _rotate(s_pts, s_splits, R, transpose=True)
    return s_pts, s_len


def _splits(lengths):
    s = np.zeros(len(lengths) + 1, np.int64)
    s[1:] = np.cumsum(lengths)
    return torch.from_numpy(s)


def batch_neighbors(queries, supports, q_lengths, s_lengths, radius, hash_table=None):
    """Dense neighbour matrix padded with the shadow index len(supports)
    (kpconv.py:2002-2034): fixed-radius search + ragged_to_dense, width =
    the largest neighbourhood.  int32 on the GPU.  ``hash_table`` (built for
    the supports at this radius) may be shared between searches."""
    return ops.fixed_radius_search_dense(supports, queries, radius, _splits(s_lengths), _splits(q_lengths),
                                         hash_table=hash_table)


# ---------------------------------------------------------------------------
# collate in two host reads per layer: every search count / subsampling count
# of a stage is queued, then their sizes come back in ONE pinned transfer
# (the reference reads each size separately: ~9 host round trips per layer)
# ---------------------------------------------------------------------------
class _Reads:
    """Device int64 slots that several collate steps fill with their sizes,
    read back in ONE pinned transfer (one buffer per device, reused: every
    read waits for its transfer before the slots are handed out again)."""
    _bufs = {}

    def __init__(self, dev):
        self.dev = dev
        key = (dev, threading.get_ident())  # per host thread (collates may run in threads)
        buf = _Reads._bufs.get(key)
        if buf is None:
            buf = _Reads._bufs[key] = torch.empty(256, dtype=torch.int64, device=dev)
        self.buf, self.used = buf, 0

    def take(self, k):
        if self.used + k > self.buf.numel():
            raise RuntimeError("collate: too many batch items for the size slots")
        off = self.used
        self.used += k
        return self.buf[off:off + k]

    def read(self):
        host = ops._pinned_slot(self.dev, self.used)
        host.copy_(self.buf[:self.used], non_blocking=True)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.dev))
        ready.synchronize()
        return host.tolist()


def _dense_begin(reads, queries, supports, q_lengths, s_lengths, radius, table=None):
    """batch_neighbors, count phase (one library call: the supports' hash
    table — built here unless ``table``, an earlier search over the same
    supports at this radius, holds it — the count, [total, long rows, width]
    into 3 device slots)."""
    return ops._layer_count(supports, queries, radius, _splits(s_lengths), _splits(q_lengths), table=table,
                            sizes=reads.take(3))


def _dense_end(x, host):
    """batch_neighbors, fill phase from the host values [total, long rows,
    width]: the rows written straight into the dense matrix padded with the
    shadow index (no CSR, no ragged_to_dense pass)."""
    _total, n_over, width = host
    if x.m == 0 or width == 0:
        return torch.full((x.m, width), x.n, dtype=torch.int32, device=x.dev)
    return ops._layer_fill_dense(x, int(width), x.n, 1 | (2 if n_over else 0))


def _subsample_begin(reads, points, lengths, sampleDl, rotations=None):
    """batch_grid_subsampling, count phase (rotation drawn here, as the reference)."""
    lengths = np.asarray(lengths, np.int64)
    splits = np.zeros(len(lengths) + 1, np.int64)
    splits[1:] = np.cumsum(lengths)
    R = random_rotations(len(lengths)) if rotations is None else np.asarray(rotations, np.float32)
    pts = _rotate(points, splits, R).contiguous()
    dev = pts.device
    lib = _lib.load()
    n, B = pts.shape[0], len(lengths)
    ws = workspace(lib.o3dml_grid_subsample_workspace_size(n, B), dev)
    out = reads.take(2 + B)
    _lib.call("o3dml_grid_subsample_count_async", ptr(pts), n, B, ptr(to_dev(splits, dev)), float(sampleDl), 0,
              ptr(out), ptr(ws), ws.numel(), stream_handle(dev))
    return pts, n, B, ws, out, R


def _subsample_end(b, host):
    """batch_grid_subsampling, fill phase from host [points, flag, lengths...]."""
    pts, n, B, ws, _, R = b
    if host[1]:
        raise RuntimeError("grid_subsample: grid too large")
    S = int(host[0])
    s_len = np.asarray(host[2:2 + B], np.int64)
    dev = pts.device
    out_p = torch.empty((S, 3), dtype=torch.float32, device=dev)
    out_l = torch.empty(B, dtype=torch.int64, device=dev)
    _lib.call("o3dml_grid_subsample_fill", ptr(pts), n, B, None, 0, None, 0, ptr(out_p), None, None, ptr(out_l),
              ptr(ws), ws.numel(), stream_handle(dev))
    s_splits = np.zeros(B + 1, np.int64)
    s_splits[1:] = np.cumsum(s_len)
    return _rotate(out_p, s_splits, R, transpose=True), s_len


def segmentation_inputs(cfg, stacked_points, stacked_features, labels, stack_lengths, neighborhood_limits=(),
                        rotations=None):
    """concat_batcher.py:186-283 on the GPU.  ``rotations`` optionally fixes
    the random grid orientation of each subsampling call (list of [B,3,3]),
    otherwise they are drawn from np.random as the reference does."""
    cfg = Config(DEFAULTS, **cfg) if not isinstance(cfg, Config) else cfg
    dev = stacked_features.device if stacked_features.is_cuda else torch.device("cuda", torch.cuda.current_device())
    stacked_points = stacked_points.to(dev).float().contiguous()
    stack_lengths = np.asarray(stack_lengths, np.int64)
    r_normal = cfg.first_subsampling_dl * cfg.conv_radius
    points, neighbors, pools, upsamples, lengths = [], [], [], [], []
    empty = torch.zeros((0, 1), dtype=torch.int32, device=dev)
    sub_i = 0

    def limit(nb, layer):
        return nb[:, :neighborhood_limits[layer]] if len(neighborhood_limits) > 0 else nb

    # the architecture as layers: (the layer's conv blocks, the block that ends it)
    layers, layer_blocks = [], []
    for block in cfg.architecture:
        if not any(t in block for t in ("pool", "strided", "global", "upsample")):
            layer_blocks.append(block)
            continue
        layers.append((layer_blocks, block))
        layer_blocks = []
        if "global" in block or "upsample" in block:
            break

    def stage1(reads, li, pts, lens, r_norm, table=None, r_table=None):
        """Layer li's conv search count and subsampling count into `reads`
        (the conv search reuses `table` when it was built over `pts` at the
        same radius).  Returns (conv handle, subsample handle, conv radius)."""
        nonlocal sub_i
        lblocks, block = layers[li]
        conv_b = sub_b = r_conv = None
        if lblocks:
            deform = any("deformable" in b for b in lblocks)
            r_conv = r_norm * cfg.deform_radius / cfg.conv_radius if deform else r_norm
            conv_b = _dense_begin(reads, pts, pts, lens, lens, r_conv, table if r_table == r_conv else None)
        if "pool" in block or "strided" in block:
            rot = None if rotations is None else rotations[sub_i]
            sub_i += 1
            sub_b = _subsample_begin(reads, pts, lens, 2 * r_norm / cfg.conv_radius, rotations=rot)
        return conv_b, sub_b, r_conv

    # Host reads: layer 0's stage 1 alone, then per pooling layer ONE read
    # for its pool / up-sampling search counts together with the next layer's
    # conv search and subsampling counts (the reference reads each size
    # separately: ~9 round trips per layer); the up-sampling search's table
    # (the subsampled points at twice the radius) serves the next layer's conv
    # search when the radii agree.
    reads = _Reads(dev)
    conv_b, sub_b, r_conv = stage1(reads, 0, stacked_points, stack_lengths, r_normal) if layers else (None,) * 3
    host, off = (reads.read(), 0) if layers else (None, 0)
    for li, (lblocks, block) in enumerate(layers):
        conv_i = _dense_end(conv_b, host[off:off + 3]) if conv_b else empty
        off += 3 if conv_b else 0
        pooling = "pool" in block or "strided" in block
        if pooling:
            pool_p, pool_b = _subsample_end(sub_b, host[off:])
            r = r_normal * cfg.deform_radius / cfg.conv_radius if "deformable" in block else r_normal
            reads = _Reads(dev)
            pb = _dense_begin(reads, pool_p, stacked_points, pool_b, stack_lengths, r,
                              conv_b if r == r_conv else None)
            ub = _dense_begin(reads, stacked_points, pool_p, stack_lengths, pool_b, 2 * r)
            nxt = (None,) * 3
            if li + 1 < len(layers):
                nxt = stage1(reads, li + 1, pool_p, pool_b, 2 * r_normal, table=ub, r_table=2 * r)
            host, off = reads.read(), 6
            pool_i = _dense_end(pb, host[0:3])
            up_i = _dense_end(ub, host[3:6])
            conv_b, sub_b, r_conv = nxt
        else:
            pool_i = empty
            pool_p = torch.zeros((0, 3), dtype=torch.float32, device=dev)
            pool_b = np.zeros((0,), np.int64)
            up_i = empty
            if li + 1 < len(layers):  # (not produced by the reference architectures)
                reads = _Reads(dev)
                conv_b, sub_b, r_conv = stage1(reads, li + 1, pool_p, pool_b, 2 * r_normal)
                host, off = reads.read(), 0
        conv_i = limit(conv_i, len(points))
        pool_i = limit(pool_i, len(points))
        if up_i.shape[0] > 0:
            up_i = limit(up_i, len(points) + 1)
        points.append(stacked_points)
        neighbors.append(conv_i)
        pools.append(pool_i)
        upsamples.append(up_i)
        lengths.append(torch.from_numpy(stack_lengths.astype(np.int32)))
        stacked_points, stack_lengths = pool_p, pool_b
        r_normal *= 2
    feats = stacked_features.to(dev).float().contiguous()
    lab = None if labels is None else torch.as_tensor(labels).to(dev).long()
    return KPConvBatch(points, neighbors, pools, upsamples, lengths, feats, lab)
