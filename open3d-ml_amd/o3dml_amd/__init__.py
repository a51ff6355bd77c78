"""o3dml_amd — MI355X-native (gfx950 HIP) implementation of Open3D-ML's
point-cloud hot path behind the ``open3d.ml.torch`` ops/layers API.

Putting ``open3d-ml_amd/`` on sys.path provides the ``open3d`` package (the
thin shim in ``open3d-ml_amd/open3d/``), so ``open3d.ml.torch.ops`` /
``.layers``, ``open3d.ml.contrib`` and ``open3d.core.nns`` resolve to this
package and reference model code runs unchanged.  ``torch.ops.open3d.*``
(TorchScript / torch.compile callers) is registered by ``o3dml_amd.torch_ops``.
"""
from . import _lib, contrib, core, layers, ops  # noqa: F401

__version__ = "0.1.0"


def library_path():
    return _lib.LIB_PATH


def register_torch_ops():
    """Register ``torch.ops.open3d.*`` (idempotent; see o3dml_amd.torch_ops)."""
    from . import torch_ops
    return torch_ops.OPS
