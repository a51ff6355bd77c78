"""Drop-in ``open3d`` namespace backed by o3dml_amd (MI355X HIP kernels).

Only the surface Open3D-ML's hot path binds to is provided:
``open3d.ml.torch.ops`` / ``.layers``, ``open3d.ml.contrib``,
``open3d.core.nns.NearestNeighborSearch``, ``open3d.core.Tensor`` and
``open3d.core.cuda.device_count`` (pointnet2_utils.py:35), plus the
``_build_config`` dict the reference reads (vis/visualizer.py:7, tests).
Put ``open3d-ml_amd/`` on sys.path (ahead of any real Open3D) to use it.

Open3D-ML itself (``open3d.ml.torch.models`` / ``pipelines`` / ...) comes
from the checkout ``OPEN3D_ML_ROOT`` names, as upstream (``_ml3d_alias``).
"""
import os as _os
import sys as _sys

from . import _ml3d_alias

if "OPEN3D_ML_ROOT" in _os.environ:
    # upstream open3d/__init__.py: the external checkout's ml3d joins sys.path
    print("Using external Open3D-ML in {}".format(_os.environ["OPEN3D_ML_ROOT"]))
    _sys.path.append(_os.environ["OPEN3D_ML_ROOT"])
_ml3d_alias.install()

from . import core, ml  # noqa: E402,F401

__version__ = "0.19.0+o3dml_amd"

_build_config = {
    "BUILD_PYTORCH_OPS": True,
    "BUILD_TENSORFLOW_OPS": False,
    "BUILD_CUDA_MODULE": True,
    "BUILD_GUI": False,
    # Open3D-ML reachable as open3d.ml.* (an OPEN3D_ML_ROOT checkout or ml3d on sys.path)
    "BUNDLE_OPEN3D_ML": _ml3d_alias.ml3d_available(),
}
