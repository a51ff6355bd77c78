"""SparseConvUnet on MI355X (reference
ml3d/torch/models/sparseconvnet.py).

The module tree (names, classes, parameter shapes) matches the reference, so
its state_dicts load unchanged; the layers are this build's SparseConv /
SparseConvTranspose (lattice rulebook + MFMA implicit GEMM, csrc/sparse_conv.hip)
and the InputLayer / OutputLayer index work stays on the GPU (the reference
round-trips the voxel maps through numpy, sparseconvnet.py:302-315).  One
forward runs inside a rulebook-cache scope, so all submanifold convolutions of
one level share one kernel map instead of rebuilding it per layer.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import ops
from . import sparse_conv as sc
from .layers import SparseConv, SparseConvTranspose
from .sparse_conv import rulebook_cache, rulebook_scope, scope_from


class BatchNormBlock(nn.Module):
    """sparseconvnet.py:240-258."""

    def __init__(self, m, eps=1e-4, momentum=0.01):
        super().__init__()
        self.bn = nn.BatchNorm1d(m, eps=eps, momentum=momentum)

    def forward(self, feat_list):
        if len(feat_list) == 1:
            return [self.bn(feat_list[0])]
        lengths = [f.shape[0] for f in feat_list]
        return list(torch.split(self.bn(torch.cat(feat_list, 0)), lengths))


def _folded_bn(block):
    """Eval-mode BatchNorm1d of a BatchNormBlock as a per-channel affine
    (scale, shift), cached until a parameter or buffer changes."""
    bn = block.bn
    key = (bn.weight._version, bn.bias._version, bn.running_mean._version, bn.running_var._version,
           bn.weight.device, bn.eps)
    if getattr(block, "_fold_key", None) != key:
        with torch.no_grad():
            scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
            block._fold = (scale.contiguous(), (bn.bias - bn.running_mean * scale).contiguous())
        block._fold_key = key
    return block._fold


def _fusable(module):
    """Eval mode without autograd: BN + ReLU go into the next conv's gather."""
    return not module.training and not torch.is_grad_enabled()


class ReLUBlock(nn.Module):
    """sparseconvnet.py:261-279."""

    def __init__(self):
        super().__init__()
        self.relu = nn.ReLU()

    def forward(self, feat_list):
        return [self.relu(f) for f in feat_list]


class LinearBlock(nn.Module):
    """sparseconvnet.py:282-293."""

    def __init__(self, a, b):
        super().__init__()
        self.linear = nn.Linear(a, b)

    def forward(self, feat_list):
        return [self.linear(f) for f in feat_list]


class InputLayer(nn.Module):
    """Voxelize at vs = 1 in [0, 40960)^3 and average the features of each voxel
    (sparseconvnet.py:296-331); returns (features, voxel positions, the voxel of
    every input point)."""

    def __init__(self, voxel_size=1.0):
        super().__init__()
        self.voxel_size = torch.Tensor([voxel_size, voxel_size, voxel_size])

    def forward(self, features, in_positions):
        dev = in_positions.device
        v = ops.voxelize(in_positions, torch.LongTensor([0, in_positions.shape[0]]), self.voxel_size,
                         torch.Tensor([0, 0, 0]), torch.Tensor([40960, 40960, 40960]))
        pidx, prs = v.voxel_point_indices, v.voxel_point_row_splits
        pos_sorted = in_positions[pidx]
        feat_sorted = features[pidx]
        count = prs[1:] - prs[:-1]
        nvox = count.shape[0]
        positions = pos_sorted[prs[:-1]]
        avg = torch.stack([ops.reduce_subarrays_sum(feat_sorted[:, c].contiguous(), prs) for c in range(3)], 1)
        avg = avg / count.unsqueeze(1)
        # voxel of every input point (points outside the range map nowhere, as
        # the reference's zero-initialised reverse map does: voxel 0)
        index_map = torch.zeros(in_positions.shape[0], dtype=torch.int64, device=dev)
        index_map[pidx] = torch.repeat_interleave(torch.arange(nvox, device=dev), count,
                                                  output_size=pidx.shape[0])  # no host read of the sum
        return avg, positions, index_map


class OutputLayer(nn.Module):
    """sparseconvnet.py:334-344."""

    def __init__(self, voxel_size=1.0):
        super().__init__()

    def forward(self, features_list, index_map_list):
        return torch.cat([f[m] for f, m in zip(features_list, index_map_list)], 0)


class SubmanifoldSparseConv(nn.Module):
    """sparseconvnet.py:347-385."""

    def __init__(self, in_channels, filters, kernel_size, use_bias=False, offset=None, normalize=False):
        super().__init__()
        if offset is None:
            offset = 0.0 if kernel_size[0] % 2 else 0.5
        self.net = SparseConv(in_channels=in_channels, filters=filters, kernel_size=kernel_size, use_bias=use_bias,
                              offset=torch.full((3,), offset, dtype=torch.float32), normalize=normalize)

    def forward(self, features_list, in_positions_list, out_positions_list=None, voxel_size=1.0):
        if out_positions_list is None:
            out_positions_list = in_positions_list
        return [self.net(f, i, o, voxel_size) for f, i, o in zip(features_list, in_positions_list,
                                                                 out_positions_list)]


class Convolution(nn.Module):
    """Stride-2 2^3 convolution onto calculate_grid (sparseconvnet.py:404-441)."""

    def __init__(self, in_channels, filters, kernel_size, use_bias=False, offset=None, normalize=False):
        super().__init__()
        if offset is None:
            offset = 0.0 if kernel_size[0] % 2 else -0.5
        self.net = SparseConv(in_channels=in_channels, filters=filters, kernel_size=kernel_size, use_bias=use_bias,
                              offset=torch.full((3,), offset, dtype=torch.float32), normalize=normalize)

    def forward(self, features_list, in_positions_list, voxel_size=1.0, out_positions_list=None):
        if out_positions_list is None:  # UNet passes the grids it computed on its side stream
            out_positions_list = [ops.calculate_grid(p) for p in in_positions_list]
        out_feat = [self.net(f, i, o, voxel_size) for f, i, o in zip(features_list, in_positions_list,
                                                                    out_positions_list)]
        return out_feat, [o / 2 for o in out_positions_list]


class DeConvolution(nn.Module):
    """sparseconvnet.py:444-482."""

    def __init__(self, in_channels, filters, kernel_size, use_bias=False, offset=None, normalize=False):
        super().__init__()
        if offset is None:
            offset = 0.0 if kernel_size[0] % 2 else -0.5
        self.net = SparseConvTranspose(in_channels=in_channels, filters=filters, kernel_size=kernel_size,
                                       use_bias=use_bias, offset=torch.full((3,), offset, dtype=torch.float32),
                                       normalize=normalize)

    def forward(self, features_list, in_positions_list, out_positions_list, voxel_size=1.0):
        return [self.net(f, i, o, voxel_size) for f, i, o in zip(features_list, in_positions_list,
                                                                 out_positions_list)]


class ConcatFeat(nn.Module):
    def forward(self, feat):
        return feat


class JoinFeat(nn.Module):
    def forward(self, feat_cat, feat):
        return [torch.cat([a, b], -1) for a, b in zip(feat_cat, feat)]


class NetworkInNetwork(nn.Module):
    def __init__(self, nIn, nOut, bias=False):
        super().__init__()
        self.linear = nn.Identity() if nIn == nOut else nn.Linear(nIn, nOut, bias=bias)

    def forward(self, inputs):
        if isinstance(self.linear, nn.Linear) and _fusable(self) and inputs and inputs[0].is_cuda:
            # eval: one HIP dense launch (csrc/dense.hip) instead of torch's
            # GEMM, whose per-call host cost (library heuristics) was ~50 us
            from .randlanet import dense_act
            w = self.linear.weight.detach()
            b = None if self.linear.bias is None else self.linear.bias.detach()
            return [dense_act(x.contiguous(), w, b) for x in inputs]
        return [self.linear(x) for x in inputs]


class ResidualBlock(nn.Module):
    """sparseconvnet.py:532-565."""

    def __init__(self, nIn, nOut):
        super().__init__()
        self.lin = NetworkInNetwork(nIn, nOut)
        self.batch_norm1 = BatchNormBlock(nIn)
        self.relu1 = ReLUBlock()
        self.sub_sparse_conv1 = SubmanifoldSparseConv(in_channels=nIn, filters=nOut, kernel_size=[3, 3, 3])
        self.batch_norm2 = BatchNormBlock(nOut)
        self.relu2 = ReLUBlock()
        self.sub_sparse_conv2 = SubmanifoldSparseConv(in_channels=nOut, filters=nOut, kernel_size=[3, 3, 3])

    def forward(self, feat_list, pos_list):
        if _fusable(self):
            pre1, pre2 = _folded_bn(self.batch_norm1), _folded_bn(self.batch_norm2)
            c1, c2 = self.sub_sparse_conv1.net, self.sub_sparse_conv2.net
            out1 = self.lin(feat_list)
            hs = [c1.forward_fused(f, p, p, 1.0, pre=pre1) for f, p in zip(feat_list, pos_list)]
            return [c2.forward_fused(h, p, p, 1.0, pre=pre2, residual=r) for h, p, r in zip(hs, pos_list, out1)]
        out1 = self.lin(feat_list)
        f = self.relu1(self.batch_norm1(feat_list))
        f = self.sub_sparse_conv1(f, pos_list)
        f = self.relu2(self.batch_norm2(f))
        out2 = self.sub_sparse_conv2(f, pos_list)
        return [a + b for a, b in zip(out1, out2)]


def _unet_layers(planes, residual, reps):
    """The reference's recursive layer list (sparseconvnet.py:585-618)."""
    layers = []

    def block(a, b):
        if residual:
            layers.append(ResidualBlock(a, b))
        else:
            layers.extend([BatchNormBlock(a), ReLUBlock(), SubmanifoldSparseConv(a, b, [3, 3, 3])])

    for _ in range(reps):
        block(planes[0], planes[0])
    if len(planes) > 1:
        layers.extend([ConcatFeat(), BatchNormBlock(planes[0]), ReLUBlock(),
                       Convolution(planes[0], planes[1], [2, 2, 2])])
        layers.extend(_unet_layers(planes[1:], residual, reps))
        layers.extend([BatchNormBlock(planes[1]), ReLUBlock(), DeConvolution(planes[1], planes[0], [2, 2, 2]),
                       JoinFeat()])
        for i in range(reps):
            block(planes[0] * (2 if i == 0 else 1), planes[0])
    return layers


def _grid_mode():
    """O3DML_SCN_GRIDS: "front" (default) computes every level's grid before
    the first convolution is queued, "side" computes each when its
    Convolution needs it on a side stream (A/B)."""
    import os
    return os.environ.get("O3DML_SCN_GRIDS", "front")


class _LevelGrids:
    """The stride-2 grid of each level (calculate_grid, then / 2) for the
    UNet's Convolutions.  calculate_grid reads its output size back to the
    host; issued on the caller's stream between the convolutions, that read
    waited for every convolution queued above it.  "front": all levels are
    computed when this object is made (before any convolution: the reads wait
    only for the grid kernels).  "side": each level when its Convolution needs
    it, on a side stream, so the read waits only for the grid kernels while
    the queued convolutions keep the GPU busy; the side stream first waits for
    the caller's stream as of construction (the input positions), each grid
    (the next level's input) is then ordered on the side stream itself, and
    the caller's stream waits for the side stream before it uses a grid."""
    _streams = {}

    def __init__(self, pos_list, n_down):
        self.dev = pos_list[0].device if pos_list and pos_list[0].is_cuda else None
        self.ready = None
        self.chain = None
        if _grid_mode() != "side" or self.dev is None:
            self.chain = []
            for _ in range(n_down):
                outs = [ops.calculate_grid(p) for p in pos_list]
                pos_list = [o / 2 for o in outs]
                self.chain.append((outs, pos_list))
            self.chain.reverse()
        else:
            self.main = torch.cuda.current_stream(self.dev)
            self.ready = torch.cuda.Event()
            self.ready.record(self.main)

    def next(self, pos_list):
        if self.chain is not None:
            return self.chain.pop()
        side = self._streams.get(self.dev)
        if side is None:
            side = self._streams[self.dev] = torch.cuda.Stream(self.dev)
        if self.ready is not None:
            side.wait_event(self.ready)
            self.ready = None
        with torch.cuda.stream(side):
            outs = [ops.calculate_grid(p) for p in pos_list]
            half = [o / 2 for o in outs]
        for t in outs + half:
            t.record_stream(self.main)  # freed blocks wait for the caller's stream
        self.main.wait_stream(side)
        return outs, half


class _FixedGrids:
    """_LevelGrids' interface over the per-level grids of a captured body:
    level l's Convolution output grid, the next level's positions = grid / 2
    computed in the body (one kernel, no extra graph input) unless given
    (halves_per_level: the plan's, same bits)."""

    def __init__(self, outs_per_level, halves_per_level=None):
        self.levels = list(outs_per_level)
        self.halves = None if halves_per_level is None else list(halves_per_level)

    def next(self, pos_list):
        outs = self.levels.pop(0)
        if self.halves is not None:
            return outs, self.halves.pop(0)
        return outs, [o / 2 for o in outs]


def _graph_mode():
    """O3DML_SCN_GRAPH: "1" replays the eval body as ONE HIP graph per size
    signature (_ScnBody), "2" as a head + tail pair with the deeper
    level grids computed on a side stream while the head replays
    (_ScnHead / _ScnTail), "3" runs the InputLayer and every level grid as
    one library call into persistent buffers the captured body reads in
    place (_ScnPlan / _ScnPlanBody; the default), "0" runs it eagerly (A/B).
    Modes 1 and 3 capture a signature the second time it is seen
    (SparseConvUnet._seen_before)."""
    return os.environ.get("O3DML_SCN_GRAPH", "3")


def _map_stream_on():
    """O3DML_SCN_MAP_STREAM: "1" (default) builds the eval plan body's kernel
    maps on a second stream (SparseConvUnet._plan_body), "0" in line (A/B)."""
    return os.environ.get("O3DML_SCN_MAP_STREAM", "1") != "0"


_MAP_STREAMS = {}


def _map_stream(dev):
    s = _MAP_STREAMS.get(dev)
    if s is None:
        s = _MAP_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def _copy_into(dst_lists, src_lists):
    for dl, sl in zip(dst_lists, src_lists):
        for dst, src in zip(dl, sl):
            dst.copy_(src)


class _ScnPlan:
    """Persistent buffers of the one-call eval plan (o3dml_scn_plan: the
    InputLayer and every level's calculate_grid) for up to `cap` points:
    voxel positions / mean features, every point's voxel, and each level's
    grid at a fixed offset, so a captured body reads them in place (no copies
    into graph inputs)."""

    def __init__(self, cap, fdim, n_levels, dev):
        from . import _lib
        from ._util import workspace
        self.cap, self.fdim, self.n_levels = cap, fdim, n_levels
        self.vpos = torch.empty((cap, 3), dtype=torch.float32, device=dev)
        self.vfeat = torch.empty((cap, fdim), dtype=torch.float32, device=dev)
        self.imap = torch.empty(cap, dtype=torch.int64, device=dev)
        self.grids = torch.empty((n_levels, cap, 3), dtype=torch.float32, device=dev)
        self.halves = torch.empty((n_levels, cap, 3), dtype=torch.float32, device=dev)
        self.ws = workspace(_lib.load().o3dml_scn_plan_workspace_size(cap), dev)
        self.sizes = np.zeros(1 + n_levels, np.int64)

    def run(self, points, features):
        from . import _lib
        from ._util import ptr, stream_handle
        n = int(points.shape[0])
        if n > self.cap:
            raise RuntimeError(f"scn plan: {n} points > capacity {self.cap}")
        _lib.call("o3dml_scn_plan", ptr(points), ptr(features), n, self.cap, self.fdim, self.n_levels, ptr(self.vpos),
                  ptr(self.vfeat), ptr(self.imap), ptr(self.grids), ptr(self.halves), self.sizes.ctypes.data,
                  ptr(self.ws), self.ws.numel(), stream_handle(points.device))
        nv = int(self.sizes[0])
        outs = [self.grids[l, :int(self.sizes[1 + l])] for l in range(self.n_levels)]
        halves = [self.halves[l, :int(self.sizes[1 + l])] for l in range(self.n_levels)]
        return n, self.vpos[:nv], self.vfeat[:nv], self.imap[:n], (outs, halves)


class _ScnPlanBody:
    """The eval body (every convolution and map, the head, the OutputLayer
    gather) captured per size signature on a _ScnPlan's buffers and replayed
    per frame right after the one-call plan — no input copies."""

    def __init__(self, model, pos, feat, imap, grids):
        dev = pos.device
        main = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):  # warm-up: lazy caches and library state outside the capture
            with rulebook_cache(defer_checks=True) as scope:
                model._plan_body(pos, feat, imap, grids)
                ok = scope.check()
                searches = scope.searches
        main.wait_stream(side)
        self.graph = None
        if not ok or searches:
            return
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            with rulebook_cache(defer_checks=True) as scope:
                self.out = model._plan_body(pos, feat, imap, grids)
                self.status = torch.cat(scope.pending) if scope.pending else None
                scope.pending.clear()


class _ScnBody:
    """The eval forward after the InputLayer and the level grids — every
    convolution with its lattice kernel map, the folded BatchNorm / ReLU
    prologues, the residual epilogues, the head — captured once per size
    signature (voxels and grid points of every level) as a HIP graph and
    replayed per frame: ~330 launches and their host cost become one replay.
    The frame's inputs (voxel positions, averaged features, the level grids)
    are copied into the graph's static buffers first; the lattice status
    words the body leaves on the device are read once after the replay (the
    eager path's scope.check)."""

    def __init__(self, model, pos_list, feat_list, outs_per_level):
        dev = pos_list[0].device
        self.pos = [p.clone() for p in pos_list]
        self.feat = [f.clone() for f in feat_list]
        self.outs = [[o.clone() for o in outs] for outs in outs_per_level]
        main = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):  # warm-up: lazy caches and library state outside the capture
            with rulebook_cache(defer_checks=True) as scope:
                model._body(self.pos, self.feat, _FixedGrids(self.outs))
                ok = scope.check()
                searches = scope.searches
        main.wait_stream(side)
        self.lattice = ok
        self.graph = None
        # off-lattice input, or a layer on the search rulebook (e.g. an empty
        # level): the caller takes the eager path
        if not ok or searches:
            return
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            with rulebook_cache(defer_checks=True) as scope:
                self.out = model._body(self.pos, self.feat, _FixedGrids(self.outs))
                self.status = torch.cat(scope.pending) if scope.pending else None
                scope.pending.clear()

    def run(self, pos_list, feat_list, outs_per_level):
        """Replay on this frame's inputs; None when a level is off the lattice."""
        for dst, src in zip(self.pos, pos_list):
            dst.copy_(src)
        for dst, src in zip(self.feat, feat_list):
            dst.copy_(src)
        for dl, sl in zip(self.outs, outs_per_level):
            for dst, src in zip(dl, sl):
                dst.copy_(src)
        self.graph.replay()
        if self.status is not None:
            st = self.status.cpu()
            if bool((st & 1).any()):
                raise RuntimeError("sparse_conv: two neighbours of one output share a kernel index")
            if bool((st & 4).any()):
                return None
        return self.out


class _ScnTail:
    """The eval body from the second Convolution on (needs level grids 1..),
    captured per grid-size signature under one _ScnHead, continuing the
    head's rulebook scope (the level-0 map the decoder's last block reuses is
    the head's); its graph also concatenates every lattice status word."""

    def __init__(self, model, head, rest):
        dev = head.pos[0].device
        self.outs = [[o.clone() for o in outs] for outs in rest]
        main = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):  # warm-up on the head's outputs of this frame, in a scratch scope
            import copy
            with rulebook_scope(scope_from(head.maps)) as scope:
                model._body_tail(copy.copy(head.state), _FixedGrids(self.outs), fresh=True)
                scope.pending[:0] = head.pending
                ok = scope.check()
                searches = scope.searches
        main.wait_stream(side)
        self.graph = None
        if not ok or searches:  # off-lattice, or a layer on the search rulebook: eager path
            return
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            with rulebook_scope(scope_from(head.maps)) as scope:
                self.out = model._body_tail(copy.copy(head.state), _FixedGrids(self.outs), fresh=True)
                pending = head.pending + scope.pending
                self.status = torch.cat(pending) if pending else None


class _ScnHead:
    """The eval body up to the second Convolution — the input convolution,
    the level-0 block, the first stride-2 Convolution (level-0 grid) and the
    level-1 block — captured once per (voxels, level-0 grid points) as a HIP
    graph.  Its replay runs while the host computes the deeper level grids
    on a side stream (each calculate_grid reads its size back: those reads
    then wait only for the grid kernels, not for the convolutions); the tail
    (_ScnTail, per deeper grid sizes) replays after them.  Inputs are copied
    into the graphs' static buffers; the lattice status words are read once
    per frame, after the tail (the eager path's scope.check)."""

    _MAX_TAILS = 4

    def __init__(self, model, pos_list, feat_list, outs0, rest):
        dev = pos_list[0].device
        self.pos = [p.clone() for p in pos_list]
        self.feat = [f.clone() for f in feat_list]
        self.outs0 = [[o.clone() for o in outs0]]
        self.tails = {}
        main = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):  # warm-up of the whole body: lazy caches and library state
            with rulebook_cache(defer_checks=True) as scope:
                st = model._body_head(self.pos, self.feat, self.outs0)
                model._body_tail(st, _FixedGrids([[o.clone() for o in outs] for outs in rest]))
                ok = scope.check()
                searches = scope.searches
        main.wait_stream(side)
        self.graph = None
        if not ok or searches:
            return
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            with rulebook_cache(defer_checks=True) as scope:
                self.state = model._body_head(self.pos, self.feat, self.outs0)
                self.maps = dict(scope.maps)
                self.pending = list(scope.pending)

    def replay(self, pos_list, feat_list, outs0):
        _copy_into([self.pos, self.feat], [pos_list, feat_list])
        _copy_into(self.outs0, [outs0])
        self.graph.replay()

    def tail(self, model, rest):
        key = tuple(tuple(int(o.shape[0]) for o in outs) for outs in rest)
        t = self.tails.pop(key, None)
        if t is None:
            t = _ScnTail(model, self, rest)
            while len(self.tails) >= self._MAX_TAILS:
                self.tails.pop(next(iter(self.tails)))
        self.tails[key] = t
        return t


_GRID_STREAMS = {}


def _grid_stream(dev):
    """One side stream per device for the deeper level grids (created once;
    O3DML_SCN_SIDE_PRIO=1: at the highest stream priority, A/B)."""
    st = _GRID_STREAMS.get(str(dev))
    if st is None:
        prio = 0
        if os.environ.get("O3DML_SCN_SIDE_PRIO", "0") == "1":
            prio = torch.cuda.Stream.priority_range()[1]
        st = _GRID_STREAMS[str(dev)] = torch.cuda.Stream(dev, priority=prio)
    return st


def _status_ok(status):
    if status is None:
        return True
    st = status.cpu()
    if bool((st & 1).any()):
        raise RuntimeError("sparse_conv: two neighbours of one output share a kernel index")
    return not bool((st & 4).any())


class UNet(nn.Module):
    """sparseconvnet.py:568-653."""

    def __init__(self, conv_block_reps, nPlanes, residual_blocks=False, downsample=(2, 2), leakiness=0):
        super().__init__()
        self.net = nn.ModuleList(_unet_layers(list(nPlanes), residual_blocks, conv_block_reps))
        self.residual_blocks = residual_blocks

    def n_down(self):
        return sum(isinstance(m, Convolution) for m in self.net)

    def split_index(self, k):
        """Index in self.net of the k-th Convolution (1-based; len(net) if
        there are fewer): a run stopped there needs only the first k - 1
        level grids."""
        seen = 0
        for j, m in enumerate(self.net):
            if isinstance(m, Convolution):
                seen += 1
                if seen == k:
                    return j
        return len(self.net)

    def begin(self, pos_list, feat_list):
        """State of a (resumable) forward: run(state, grids, stop) advances it."""
        import types
        return types.SimpleNamespace(j=0, pos_list=pos_list, feat_list=feat_list, conv_pos=[], conv_out=[],
                                     concat_feat=[], pre=None)

    def map_schedule(self, pos, outs, halves):
        """The (layer, input positions, output positions) of every kernel map
        the forward builds, in the order it needs them, for one batch element
        whose level grids and their halves are given (the eval plan's)."""
        sched, conv_pos, conv_out, p, lvl = [], [], [], pos, 0
        for m in self.net:
            if isinstance(m, ResidualBlock):
                sched.append((m.sub_sparse_conv1.net, p, p))
                sched.append((m.sub_sparse_conv2.net, p, p))
            elif isinstance(m, SubmanifoldSparseConv):
                sched.append((m.net, p, p))
            elif isinstance(m, Convolution):
                conv_pos.append(p)
                conv_out.append(outs[lvl])
                sched.append((m.net, p, outs[lvl]))
                p = halves[lvl]
                lvl += 1
            elif isinstance(m, DeConvolution):
                sched.append((m.net, conv_out.pop(), conv_pos[-1]))
                p = conv_pos.pop()
        return sched

    def forward(self, pos_list, feat_list, grids=None):
        if grids is None:
            grids = _LevelGrids(pos_list, self.n_down())
        st = self.begin(pos_list, feat_list)
        self.run(st, grids)
        return st.feat_list

    def run(self, st, grids, stop=None):
        # conv_out: each Convolution's output grid in the fine level's units —
        # the DeConvolution's input positions (= 2 x the coarse positions,
        # exactly), the same tensor, so the DeConvolution's kernel map is
        # derived from the Convolution's (sparse_conv._transpose_of_cached)
        mods = list(self.net)
        stop = len(mods) if stop is None else stop
        fuse = _fusable(self)
        conv_pos, conv_out, concat_feat = st.conv_pos, st.conv_out, st.concat_feat
        pos_list, feat_list, pre = st.pos_list, st.feat_list, st.pre
        # pending folded BN + ReLU (eval): applied by the next conv's gather
        for j in range(st.j, stop):
            m = mods[j]
            if fuse and isinstance(m, BatchNormBlock) and j + 2 < len(mods) and \
                    isinstance(mods[j + 1], ReLUBlock) and \
                    isinstance(mods[j + 2], (SubmanifoldSparseConv, Convolution, DeConvolution)):
                pre = _folded_bn(m)
                continue
            if pre is not None and isinstance(m, ReLUBlock):
                continue
            if pre is not None:
                if isinstance(m, SubmanifoldSparseConv):
                    feat_list = [m.net.forward_fused(f, p, p, 1.0, pre=pre) for f, p in zip(feat_list, pos_list)]
                elif isinstance(m, Convolution):
                    conv_pos.append(pos_list)
                    outs, half = grids.next(pos_list)
                    conv_out.append(outs)
                    feat_list = [m.net.forward_fused(f, p, o, 1.0, pre=pre)
                                 for f, p, o in zip(feat_list, pos_list, outs)]
                    pos_list = half
                else:  # DeConvolution
                    feat_list = [m.net.forward_fused(f, c, o, 1.0, pre=pre)
                                 for f, c, o in zip(feat_list, conv_out.pop(), conv_pos[-1])]
                    pos_list = conv_pos.pop()
                pre = None
                continue
            if isinstance(m, (BatchNormBlock, ReLUBlock)):
                feat_list = m(feat_list)
            elif isinstance(m, (ResidualBlock, SubmanifoldSparseConv)):
                feat_list = m(feat_list, pos_list)
            elif isinstance(m, Convolution):
                conv_pos.append(pos_list)
                outs, half = grids.next(pos_list)
                conv_out.append(outs)
                feat_list, _ = m(feat_list, pos_list, out_positions_list=outs)
                pos_list = half
            elif isinstance(m, DeConvolution):
                feat_list = m(feat_list, conv_out.pop(), conv_pos[-1])
                pos_list = conv_pos.pop()
            elif isinstance(m, ConcatFeat):
                concat_feat.append(m(feat_list))
            elif isinstance(m, JoinFeat):
                feat_list = m(concat_feat.pop(), feat_list)
            else:
                raise Exception("Unknown module {}".format(m))
        st.j, st.pos_list, st.feat_list, st.pre = stop, pos_list, feat_list, pre
        return st


class SparseConvUnet(nn.Module):
    """sparseconvnet.py:13-93 (model part; data preprocessing stays the caller's).
    forward(inputs) takes an object with .point / .feat lists and .batch_lengths
    like the reference ConcatBatcher output and returns per-point logits."""

    def __init__(self, name="SparseConvUnet", device="cuda", multiplier=16, voxel_size=0.05, conv_block_reps=1,
                 residual_blocks=False, in_channels=3, num_classes=20, grid_size=4096, **kwargs):
        super().__init__()
        self.multiplier = multiplier
        self.input_layer = InputLayer()
        self.sub_sparse_conv = SubmanifoldSparseConv(in_channels=in_channels, filters=multiplier,
                                                     kernel_size=[3, 3, 3])
        self.unet = UNet(conv_block_reps, [multiplier * i for i in range(1, 8)], residual_blocks)
        self.batch_norm = BatchNormBlock(multiplier)
        self.relu = ReLUBlock()
        self.linear = LinearBlock(multiplier, num_classes)
        self.output_layer = OutputLayer()

    _MAX_GRAPHS = 4  # captured bodies kept per model (size signatures, LRU)

    def forward(self, inputs):
        mode = _graph_mode()
        if mode != "0" and not self.training and not torch.is_grad_enabled() and len(inputs.point) and \
                inputs.point[0].is_cuda:
            if mode == "3":
                out = self._forward_plan(inputs)
            else:
                out = self._forward_graph(inputs) if mode == "2" else self._forward_graph_single(inputs)
            if out is not None:
                return out
        # lattice checks of all levels are read back once at the end; a
        # non-lattice input (never produced by the reference preprocess) is
        # recomputed with per-layer checks and the search rulebook
        with rulebook_cache(defer_checks=True) as scope:
            out = self._forward(inputs)
            ok = scope.check()
        if ok:
            return out
        with rulebook_cache():
            return self._forward(inputs)

    def _inputs(self, inputs):
        pos_list, feat_list, index_maps = [], [], []
        for i in range(len(inputs.batch_lengths)):
            f, p, m = self.input_layer(inputs.feat[i], inputs.point[i])
            pos_list.append(p)
            feat_list.append(f)
            index_maps.append(m)
        return pos_list, feat_list, index_maps

    def _body(self, pos_list, feat_list, grids):
        """Everything between the InputLayer (+ level grids) and the head."""
        feat_list = self.sub_sparse_conv(feat_list, pos_list, voxel_size=1.0)
        return self.unet(pos_list, feat_list, grids=grids)

    def _head(self, feat_list, index_maps):
        """BatchNorm + ReLU, the Linear and the OutputLayer gather.  Eval
        without autograd, one batch element: the folded BN + ReLU as one
        addcmul + relu, then the Linear over the gathered rows in one dense
        launch (randlanet.dense_act with a row index: logits of every point
        straight from its voxel's features) — every eval path (eager and
        captured) runs this same head."""
        lin = self.linear.linear
        if _fusable(self) and len(feat_list) == 1 and feat_list[0].is_cuda and isinstance(lin, nn.Linear):
            from .randlanet import dense_act
            s, t = _folded_bn(self.batch_norm)
            y = torch.addcmul(t, feat_list[0], s).relu_()
            return dense_act(None, lin.weight.detach(), None if lin.bias is None else lin.bias.detach(), a2=y,
                             a2_index=index_maps[0])
        feat_list = self.relu(self.batch_norm(feat_list))
        return self.output_layer(self.linear(feat_list), index_maps)

    def _body_head(self, pos_list, feat_list, outs0):
        """The body up to the second Convolution (needs the level-0 grid only)."""
        feat_list = self.sub_sparse_conv(feat_list, pos_list, voxel_size=1.0)
        st = self.unet.begin(pos_list, feat_list)
        return self.unet.run(st, _FixedGrids(outs0), stop=self.unet.split_index(2))

    def _body_tail(self, st, grids, fresh=False):
        """The rest of the body from a _body_head state.  fresh: st is a
        shallow copy whose lists must not be shared with the head's."""
        if fresh:
            st.conv_pos, st.conv_out, st.concat_feat = list(st.conv_pos), list(st.conv_out), list(st.concat_feat)
        self.unet.run(st, grids)
        return st.feat_list

    def _param_key(self):
        """(address, version) of every parameter and buffer: a captured body
        is only replayed on the weights it was captured with.  The tensor list
        is kept (walking the module tree costs ~1 ms per frame) and dropped by
        _apply (.to / .cuda / .float replace the tensors)."""
        ts = self.__dict__.get("_o3dml_state_tensors")
        if ts is None:
            ts = self.__dict__["_o3dml_state_tensors"] = list(self.parameters()) + list(self.buffers())
        return tuple((t.data_ptr(), t._version) for t in ts)

    _SEEN = 16  # size signatures remembered for the capture-on-second-sighting policy

    def _seen_before(self, key):
        """Capture policy of the graph modes: a size signature is captured the
        second time it is seen, so a stream of frames that never repeat a size
        (every scan of a dataset differs) pays no capture, only the eager body;
        a repeated frame (the benchmark, a fixed-size crop) replays."""
        seen = self.__dict__.setdefault("_o3dml_scn_seen", {})
        hit = seen.pop(key, None) is not None
        seen[key] = True
        while len(seen) > self._SEEN:
            seen.pop(next(iter(seen)))
        return hit

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_o3dml_state_tensors", None)
        self.__dict__.pop("_o3dml_scn_bodies", None)
        self.__dict__.pop("_o3dml_scn_single", None)
        self.__dict__.pop("_o3dml_scn_plan", None)
        self.__dict__.pop("_o3dml_scn_plan_bodies", None)
        self.__dict__.pop("_o3dml_scn_seen", None)
        return super()._apply(fn, *args, **kwargs)

    def _forward_graph(self, inputs):
        """Eval forward with the body replayed from captured graphs (_ScnHead /
        _ScnTail): the InputLayer and the level-0 grid run eagerly, the head
        replays while the deeper grids are computed on a side stream, then the
        tail.  None when the input is off the voxel lattice (the caller
        recomputes eagerly)."""
        pos_list, feat_list, index_maps = self._inputs(inputs)
        n_down = self.unet.n_down()
        if n_down < 2:
            return None
        outs0 = [ops.calculate_grid(x) for x in pos_list]
        dev = pos_list[0].device
        key = (str(dev), tuple(int(x.shape[0]) for x in pos_list), tuple(int(o.shape[0]) for o in outs0),
               self._param_key())
        heads = self.__dict__.setdefault("_o3dml_scn_bodies", {})
        head = heads.pop(key, None)
        fresh = head is None

        def deeper(outs):
            rest, p = [], [o / 2 for o in outs]
            for _ in range(n_down - 1):
                o = [ops.calculate_grid(x) for x in p]
                rest.append(o)
                p = [x / 2 for x in o]
            return rest

        if fresh:  # first frame of this signature: grids first, then the captures
            rest = deeper(outs0)
            head = _ScnHead(self, pos_list, feat_list, outs0, rest)
            while len(heads) >= self._MAX_GRAPHS:
                heads.pop(next(iter(heads)))
        heads[key] = head
        if head.graph is None:
            return None
        main = torch.cuda.current_stream(dev)
        grids_in = torch.cuda.Event()
        grids_in.record(main)  # the level-0 grid is ready (before the head's replay is queued)
        head.replay(pos_list, feat_list, outs0)
        if not fresh:
            # the deeper grids on a side stream while the head replays: each
            # size read waits only for the grid kernels
            side = _grid_stream(dev)
            side.wait_event(grids_in)
            with torch.cuda.stream(side):
                rest = deeper(outs0)
            for outs in rest:
                for t in outs:
                    t.record_stream(main)
            main.wait_stream(side)
        tail = head.tail(self, rest)
        if tail.graph is None:
            return None
        _copy_into(tail.outs, rest)
        tail.graph.replay()
        if not _status_ok(tail.status):
            return None
        return self._head(tail.out, index_maps)

    def _plan_body(self, pos, feat, imap, grids):
        """The eval body on the plan's buffers.  With O3DML_SCN_MAP_STREAM (default
        1) every kernel map after the first is built ahead on a second stream
        (sparse_conv.prefetch_lattice_map: the lattice maps, their tile orders,
        the derived transpose maps), one more after each convolution's GEMM
        launch (scope.pump), each convolution waiting only for its own map's event:
        the map builds run beside the GEMM chain, and a captured graph holds the
        two branches with their nodes interleaved in launch order (a graph is
        dispatched node by node in that order)."""
        outs, halves = grids
        dev = pos.device
        side = None
        scope = sc.active_scope()
        if _map_stream_on() and not torch.is_grad_enabled() and scope is not None:
            sched = [(self.sub_sparse_conv.net, pos, pos)] + self.unet.map_schedule(pos, outs, halves)
            sched[0][0].prefetch_map(pos, pos, 1.0)  # the first map is needed at once: on this stream
            main = torch.cuda.current_stream(dev)
            side = _map_stream(dev)
            side.wait_stream(main)
            scope.ahead_stream = side
            scope.ahead.extend((lambda l=l, i=i, o=o: l.prefetch_map(i, o, 1.0)) for l, i, o in sched[1:])
        out = self._body([pos], [feat], _FixedGrids([[o] for o in outs], [[h] for h in halves]))
        if side is not None:
            scope.ahead.clear()
            torch.cuda.current_stream(dev).wait_stream(side)  # join (a capture must end on one stream)
        return self._head(out, [imap])

    _PLAN_STEP = 8192  # plan buffer capacity granularity (points)

    def _forward_plan(self, inputs):
        """Eval forward as the one-call plan (o3dml_scn_plan: InputLayer +
        every level grid, one host read per size, no Python between the
        launches) and the body replayed from a graph captured on the plan's
        buffers (_ScnPlanBody).  One batch element; None when the input is off
        the voxel lattice (the caller recomputes eagerly) or batched."""
        if len(inputs.batch_lengths) != 1:
            return self._forward_graph_single(inputs)
        pts = inputs.point[0]
        feats = inputs.feat[0]
        if pts.dtype != torch.float32 or feats.dtype != torch.float32 or pts.dim() != 2 or pts.shape[1] != 3:
            return self._forward_graph_single(inputs)
        pts, feats = pts.contiguous(), feats.contiguous()
        dev = pts.device
        n = int(pts.shape[0])
        cap = max(self._PLAN_STEP, -(-n // self._PLAN_STEP) * self._PLAN_STEP)
        pk = (str(dev), cap, int(feats.shape[1]))
        plan = self.__dict__.get("_o3dml_scn_plan")
        if plan is None or plan[0] != pk:
            plan = (pk, _ScnPlan(cap, int(feats.shape[1]), self.unet.n_down(), dev))
            self.__dict__["_o3dml_scn_plan"] = plan
            self.__dict__.pop("_o3dml_scn_plan_bodies", None)  # they read the old buffers
        plan = plan[1]
        n, pos, feat, imap, grids = plan.run(pts, feats)
        outs = grids[0]
        if any(o.shape[0] == 0 for o in outs):
            return None  # an empty level: the eager path (search rulebook)
        key = (n, pos.shape[0], tuple(o.shape[0] for o in outs), self._param_key())
        bodies = self.__dict__.setdefault("_o3dml_scn_plan_bodies", {})
        body = bodies.pop(key, None)
        if body is None:
            if not self._seen_before(("plan",) + key):  # first sighting: the body eagerly on the plan's buffers
                with rulebook_cache(defer_checks=True) as scope:
                    out = self._plan_body(pos, feat, imap, grids)
                    return out if scope.check() else None
            body = _ScnPlanBody(self, pos, feat, imap, grids)
            while len(bodies) >= self._MAX_GRAPHS:
                bodies.pop(next(iter(bodies)))
        bodies[key] = body
        if body.graph is None:
            return None
        body.graph.replay()
        if not _status_ok(body.status):
            return None
        return body.out.clone()

    def _forward_graph_single(self, inputs):
        """Eval forward with the body replayed from a captured graph (_ScnBody):
        the InputLayer and the level grids (whose sizes the host reads) run
        eagerly, then the body of their size signature replays.  None when the
        input is off the voxel lattice (the caller recomputes eagerly)."""
        pos_list, feat_list, index_maps = self._inputs(inputs)
        outs_per_level, p = [], pos_list
        for _ in range(self.unet.n_down()):
            outs = [ops.calculate_grid(x) for x in p]
            outs_per_level.append(outs)
            p = [o / 2 for o in outs]
        key = (str(pos_list[0].device), tuple(int(x.shape[0]) for x in pos_list),
               tuple(tuple(int(o.shape[0]) for o in outs) for outs in outs_per_level), self._param_key())
        bodies = self.__dict__.setdefault("_o3dml_scn_single", {})
        body = bodies.pop(key, None)
        if body is None:
            if not self._seen_before(("single",) + key):  # first sighting: eagerly
                with rulebook_cache(defer_checks=True) as scope:
                    out = self._body(pos_list, feat_list, _FixedGrids(outs_per_level))
                    if not scope.check():
                        return None
                return self._head(out, index_maps)
            body = _ScnBody(self, pos_list, feat_list, outs_per_level)
            while len(bodies) >= self._MAX_GRAPHS:
                bodies.pop(next(iter(bodies)))  # least recently used first
        bodies[key] = body  # most recently used last
        if body.graph is None:
            return None
        out = body.run(pos_list, feat_list, outs_per_level)
        if out is None:
            return None
        return self._head(out, index_maps)

    def _forward(self, inputs):
        pos_list, feat_list, index_maps = [], [], []
        for i in range(len(inputs.batch_lengths)):
            f, p, m = self.input_layer(inputs.feat[i], inputs.point[i])
            pos_list.append(p)
            feat_list.append(f)
            index_maps.append(m)
        grids = _LevelGrids(pos_list, self.unet.n_down())  # before the first convolution is queued
        feat_list = self.sub_sparse_conv(feat_list, pos_list, voxel_size=1.0)
        feat_list = self.unet(pos_list, feat_list, grids=grids)
        return self._head(feat_list, index_maps)
