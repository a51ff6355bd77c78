"""Drop-in for ``open3d.ml.contrib.subsample`` / ``subsample_batch``
(KPConv grid subsampling).  numpy in, numpy out, as the
reference calls them (dataprocessing.py:33-49, kpconv.py:2099-2155); the
computation runs on the GPU (ops.grid_subsample)."""
import numpy as np
import torch

from . import ops


def _run(points, batches, features, classes, sampleDl, max_p):
    pts = torch.from_numpy(np.ascontiguousarray(points, dtype=np.float32))
    feat = None if features is None else torch.from_numpy(
        np.ascontiguousarray(np.asarray(features, np.float32).reshape(len(points), -1)))
    cls = None
    if classes is not None:
        cls = torch.from_numpy(np.ascontiguousarray(np.asarray(classes, np.int32).reshape(len(points), -1)))
    return ops.grid_subsample(pts, torch.from_numpy(np.asarray(batches, np.int64)), float(sampleDl),
                              features=feat, classes=cls, max_p=int(max_p))


def subsample(points, features=None, classes=None, sampleDl=0.1, verbose=0):
    """Grid subsampling (barycentres) -> points[, features][, classes]."""
    points = np.asarray(points, np.float32)
    out = _run(points, [len(points)], features, classes, sampleDl, 0)
    res = [out.points.numpy()]
    if features is not None:
        res.append(out.features.numpy())
    if classes is not None:
        c = out.classes.numpy()
        res.append(c.reshape(-1) if np.asarray(classes).ndim == 1 else c)
    return res[0] if len(res) == 1 else tuple(res)


def subsample_batch(points, batches, features=None, classes=None, sampleDl=0.1, method="barycenters", max_p=0,
                    verbose=0):
    """Per-batch-element grid subsampling -> (points, lengths int32[, features][, classes])."""
    if method != "barycenters":
        raise RuntimeError(f"subsample_batch: unsupported method {method!r}")
    points = np.asarray(points, np.float32)
    out = _run(points, batches, features, classes, sampleDl, max_p)
    res = [out.points.numpy(), out.lengths.numpy().astype(np.int32)]
    if features is not None:
        res.append(out.features.numpy())
    if classes is not None:
        c = out.classes.numpy()
        res.append(c.reshape(-1) if np.asarray(classes).ndim == 1 else c)
    return tuple(res)
