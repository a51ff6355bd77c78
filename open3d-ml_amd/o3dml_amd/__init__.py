"""o3dml_amd — MI355X-native (gfx950 HIP) implementation of Open3D-ML's
point-cloud hot path behind the ``open3d.ml.torch`` ops/layers API.

``import o3dml_amd.open3d_shim; o3dml_amd.open3d_shim.install()`` (or putting
``open3d-ml_amd/`` on sys.path, which provides the ``open3d`` package) makes
``open3d.ml.torch.ops`` / ``.layers``, ``open3d.ml.contrib`` and
``open3d.core.nns`` resolve to this package, so reference model code runs
unchanged.
"""
from . import _lib, contrib, core, layers, ops  # noqa: F401

__version__ = "0.1.0"


def library_path():
    return _lib.LIB_PATH
