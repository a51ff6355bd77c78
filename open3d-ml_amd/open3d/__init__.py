"""Drop-in ``open3d`` namespace backed by o3dml_amd (MI355X HIP kernels).

Only the surface Open3D-ML's hot path binds to is provided:
``open3d.ml.torch.ops`` / ``.layers``, ``open3d.ml.contrib``,
``open3d.core.nns.NearestNeighborSearch``, ``open3d.core.Tensor`` and
``open3d.core.cuda.device_count`` (pointnet2_utils.py:35), plus the
``_build_config`` dict the reference reads (vis/visualizer.py:7, tests).
Put ``open3d-ml_amd/`` on sys.path (ahead of any real Open3D) to use it.
"""
from . import core, ml  # noqa: F401

__version__ = "0.19.0+o3dml_amd"

_build_config = {
    "BUILD_PYTORCH_OPS": True,
    "BUILD_TENSORFLOW_OPS": False,
    "BUILD_CUDA_MODULE": True,
    "BUILD_GUI": False,
    "BUNDLE_OPEN3D_ML": False,
}
