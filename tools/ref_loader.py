"""Import the reference's Python (ml3d) in THIS container for golden-fixture
generation only (never shipped, never run on the GPU box).

Open3D and a few third-party modules are absent, so
in-memory stand-ins are registered before ``ml3d`` is imported:
  * ``open3d.ml.torch.ops`` / ``.layers`` / ``open3d.ml.contrib`` /
    ``open3d.core.nns`` backed by the CPU oracle (oracle/oracle.py);
  * ``addict.Dict`` and ``torch.utils.tensorboard`` minimal stubs.
The models bind these names at import time (kpconv.py:11-13,
sparseconvnet.py:9-10, point_pillars.py:30, dataprocessing.py:3,6).
"""
import os
import sys
import types
from collections import namedtuple

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


class _Dict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        for k, v in list(self.items()):
            if isinstance(v, dict) and not isinstance(v, _Dict):
                self[k] = _Dict(v)


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


# ---- oracle-backed ops with the Open3D signatures -------------------------
_FRS = namedtuple("fixed_radius_search", ["neighbors_index", "neighbors_row_splits", "neighbors_distance"])
_VOX = namedtuple("voxelize", ["voxel_coords", "voxel_point_indices", "voxel_point_row_splits",
                               "voxel_batch_splits"])


class FixedRadiusSearch:
    def __init__(self, metric="L2", ignore_query_point=False, return_distances=False, **kw):
        self.metric, self.ignore, self.ret = metric, ignore_query_point, return_distances

    def __call__(self, points, queries, radius, points_row_splits=None, queries_row_splits=None,
                 hash_table_size_factor=1 / 64, hash_table=None):
        i, rs, d = O.fixed_radius_search(_np(points), _np(queries), float(radius),
                                         None if points_row_splits is None else _np(points_row_splits),
                                         None if queries_row_splits is None else _np(queries_row_splits),
                                         metric=self.metric, ignore_query_point=self.ignore,
                                         return_distances=self.ret)
        return _FRS(torch.from_numpy(i), torch.from_numpy(rs), torch.from_numpy(d))


def ragged_to_dense(values, row_splits, out_col_size, default_value):
    v = _np(values)
    return torch.from_numpy(O.ragged_to_dense(v, _np(row_splits), int(out_col_size),
                                              _np(default_value).astype(v.dtype)))


def voxelize(points, row_splits, voxel_size, points_range_min, points_range_max,
             max_points_per_voxel=2**63 - 1, max_voxels=2**63 - 1):
    r = O.voxelize(_np(points), _np(row_splits), _np(voxel_size), _np(points_range_min),
                   _np(points_range_max), int(max_points_per_voxel), int(max_voxels))
    return _VOX(*[torch.from_numpy(x) for x in r])


def reduce_subarrays_sum(values, row_splits):
    v = _np(values)
    if v.dtype == np.float64:  # float64 runs of the reference (the truth fp32 results are held to)
        rs = _np(row_splits).astype(np.int64)
        out = np.zeros(len(rs) - 1, np.float64)
        nz = rs[1:] > rs[:-1]
        out[nz] = np.add.reduceat(v, rs[:-1][nz]) if v.size else 0.0
        return torch.from_numpy(out)
    return torch.from_numpy(O.reduce_subarrays_sum(v, _np(row_splits)))


class _SparseConvStub(torch.nn.Module):
    """Open3D layers.SparseConv restated on the oracle (CPU, forward only):
    Linf fixed-radius neighbours of out_pos - offset*vs (radius k*vs/2), kernel
    index per pair, oracle sparse_conv (+ bias).  Parameters kernel / bias /
    offset as the layer's state_dict."""
    _mirror, _sign = False, 1.0

    def __init__(self, in_channels, filters, kernel_size, activation=None, use_bias=True, normalize=False,
                 offset=None, **kw):
        super().__init__()
        self.kernel_size = list(kernel_size)
        if offset is None:
            offset = torch.zeros(3)
        self.offset = torch.nn.Parameter(torch.as_tensor(offset, dtype=torch.float32), requires_grad=False)
        self.kernel = torch.nn.Parameter(torch.zeros(*self.kernel_size, in_channels, filters))
        self.bias = torch.nn.Parameter(torch.zeros(filters)) if use_bias else None
        self.normalize = normalize
        self.activation = activation

    def forward(self, inp_features, inp_positions, out_positions, voxel_size, *a, **kw):
        vs = float(voxel_size)
        ip, op = _np(inp_positions).astype(np.float32), _np(out_positions).astype(np.float32)
        q = (op - self._sign * _np(self.offset) * vs).astype(np.float32)
        idx, rs, _ = O.fixed_radius_search(ip, q, 0.5 * vs * self.kernel_size[0], metric="Linf")
        kid = O.kernel_index(ip, q, idx, rs, self.kernel_size, vs, mirror=self._mirror)
        if inp_features.dtype == torch.float64:  # float64 run: the same rulebook, float64 sums
            K = int(np.prod(self.kernel_size))
            W = self.kernel.detach().reshape(K, self.kernel.shape[-2], self.kernel.shape[-1]).double()
            n_out = len(rs) - 1
            o = torch.repeat_interleave(torch.arange(n_out), torch.from_numpy(np.diff(rs)))
            x = inp_features.detach()[torch.from_numpy(idx).long()]
            contrib = torch.einsum("pc,pcd->pd", x, W[torch.from_numpy(kid).long()])
            out = torch.zeros((n_out, W.shape[-1]), dtype=torch.float64).index_add_(0, o, contrib)
            if self.normalize:
                cnt = torch.from_numpy(np.diff(rs)).double().clamp(min=1)
                out = out / cnt[:, None]
        else:
            out = torch.from_numpy(O.sparse_conv(_np(self.kernel), _np(inp_features), idx, kid, rs,
                                                 normalize=self.normalize))
        if self.bias is not None:
            out = out + self.bias.detach()
        return self.activation(out) if self.activation else out


class _SparseConvTransposeStub(_SparseConvStub):
    _mirror, _sign = True, -1.0


class _NNS:
    def __init__(self, t):
        self.pts = t.numpy() if hasattr(t, "numpy") else np.asarray(t)

    def knn_index(self):
        return True

    def knn_search(self, q, k):
        q = q.numpy() if hasattr(q, "numpy") else np.asarray(q)
        i, _, d = O.knn_search(self.pts, q, int(k), return_distances=True, index_dtype=np.int64)
        T = types.SimpleNamespace
        return T(numpy=lambda: i.reshape(len(q), k)), T(numpy=lambda: d.reshape(len(q), k))


def install():
    if "ml3d" in sys.modules:
        return
    _mod("addict", Dict=_Dict)
    o3d = _mod("open3d")
    o3d._build_config = {"BUILD_GUI": False, "BUILD_PYTORCH_OPS": True, "BUILD_TENSORFLOW_OPS": False}
    o3d.geometry = types.SimpleNamespace()
    core = _mod("open3d.core")
    core.cuda = types.SimpleNamespace(device_count=lambda: 0)
    core.nns = types.SimpleNamespace(NearestNeighborSearch=_NNS)
    core.Tensor = types.SimpleNamespace(from_numpy=lambda a: types.SimpleNamespace(numpy=lambda: a))
    o3d.core = core
    ml = _mod("open3d.ml")
    o3d.ml = ml
    contrib = _mod("open3d.ml.contrib", subsample=O.subsample, subsample_batch=O.subsample_batch)
    contrib.iou_bev_cpu = contrib.iou_3d_cpu = None
    ml.contrib = contrib
    mt = _mod("open3d.ml.torch")
    ops = _mod("open3d.ml.torch.ops", voxelize=voxelize, ragged_to_dense=ragged_to_dense,
               reduce_subarrays_sum=reduce_subarrays_sum)
    for n in ["knn_search", "nms", "roi_pool", "trilinear_devoxelize_forward", "trilinear_devoxelize_backward",
              "furthest_point_sampling", "three_nn", "three_interpolate", "three_interpolate_grad", "ball_query"]:
        setattr(ops, n, None)
    lay = _mod("open3d.ml.torch.layers", FixedRadiusSearch=FixedRadiusSearch, SparseConv=_SparseConvStub,
               SparseConvTranspose=_SparseConvTransposeStub)
    mt.ops, mt.layers = ops, lay
    ml.torch = mt
    _mod("open3d.visualization")
    _mod("open3d.visualization.tensorboard_plugin", summary=None)
    _mod("torch.utils.tensorboard", SummaryWriter=None)
    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
