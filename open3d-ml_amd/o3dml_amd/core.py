"""Minimal ``open3d.core`` surface used on the hot path:
``Tensor.from_numpy(...)`` / ``.numpy()``, ``nns.NearestNeighborSearch`` with
``knn_index()`` / ``knn_search(query, k)`` (dataprocessing.py:99-101) and
``fixed_radius_index(r)`` / ``fixed_radius_search(query, r)``, and
``cuda.device_count()`` (pointnet2_utils.py:35).  Searches run on the GPU."""
import types

import numpy as np
import torch

from . import ops


class Dtype:
    Float32 = "Float32"
    Float64 = "Float64"
    Int32 = "Int32"
    Int64 = "Int64"


class Device:
    def __init__(self, spec="CPU:0"):
        self.spec = spec

    def __repr__(self):
        return self.spec


class Tensor:
    """Thin wrapper over a torch tensor with Open3D's numpy interop."""

    def __init__(self, data, dtype=None, device=None):
        if isinstance(data, Tensor):
            data = data._t
        self._t = data if isinstance(data, torch.Tensor) else torch.as_tensor(np.asarray(data))

    @staticmethod
    def from_numpy(arr):
        return Tensor(torch.from_numpy(np.ascontiguousarray(arr)))

    def numpy(self):
        return self._t.detach().cpu().numpy()

    def to_torch(self):
        return self._t

    @property
    def shape(self):
        return tuple(self._t.shape)

    def __len__(self):
        return self._t.shape[0]

    def __repr__(self):
        return f"Tensor({self._t!r})"


def _as_torch(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.from_numpy(np.ascontiguousarray(x))


class NearestNeighborSearch:
    """open3d.core.nns.NearestNeighborSearch (kNN and fixed-radius paths).
    The dataset is staged on the GPU once at construction."""

    def __init__(self, dataset_points, index_dtype=None):
        pts = _as_torch(dataset_points)
        if pts.dtype != torch.float32:
            pts = pts.float()
        from ._util import gpu_device
        self._dev = gpu_device(pts)
        self._pts = pts.to(self._dev).contiguous()
        self._radius = None

    def knn_index(self):
        return True

    def fixed_radius_index(self, radius=None):
        self._radius = radius
        return True

    def hybrid_index(self, radius=None):
        self._radius = radius
        return True

    def knn_search(self, query_points, knn):
        """-> (indices Int64 [Nq, k], squared distances Float32 [Nq, k]).
        Rows hold min(k, N) neighbours; requires N >= k for a dense result."""
        q = _as_torch(query_points)
        if q.dtype != torch.float32:
            q = q.float()
        qd = q.to(self._dev).contiguous()
        n, m = self._pts.shape[0], qd.shape[0]
        if n < knn:
            raise RuntimeError(f"knn_search: k={knn} exceeds the number of dataset points {n}")
        res = ops.knn_search(self._pts, qd, int(knn), torch.LongTensor([0, n]), torch.LongTensor([0, m]),
                             index_dtype=torch.int64, return_distances=True)
        idx = res.neighbors_index.reshape(m, knn)
        dist = res.neighbors_distance.reshape(m, knn)
        return Tensor(idx.cpu()), Tensor(dist.cpu())

    def fixed_radius_search(self, query_points, radius=None, sort=True):
        """-> (indices Int64 [P], squared distances Float32 [P], row splits Int64 [Nq+1]).
        sort=True (Open3D's default) orders every row by ascending distance,
        ties in the canonical (bucket, id) order; sort=False keeps that order."""
        r = self._radius if radius is None else radius
        q = _as_torch(query_points).float().to(self._dev).contiguous()
        res = ops.fixed_radius_search(self._pts, q, float(r), index_dtype=torch.int64, return_distances=True)
        idx, dist, rs = res.neighbors_index, res.neighbors_distance, res.neighbors_row_splits
        if sort and idx.numel():
            # rows by ascending distance: a stable sort by distance, then a
            # stable sort by row keeps each row's distance order (and ties)
            row = torch.repeat_interleave(torch.arange(rs.numel() - 1, device=rs.device), rs[1:] - rs[:-1])
            o = torch.sort(dist, stable=True).indices
            o = o[torch.sort(row[o], stable=True).indices]
            idx, dist = idx[o], dist[o]
        return Tensor(idx.cpu()), Tensor(dist.cpu()), Tensor(rs.cpu())


nns = types.SimpleNamespace(NearestNeighborSearch=NearestNeighborSearch)


def _device_count():
    return torch.cuda.device_count()


cuda = types.SimpleNamespace(device_count=_device_count, is_available=lambda: torch.cuda.is_available())
