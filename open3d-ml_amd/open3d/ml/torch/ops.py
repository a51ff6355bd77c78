"""open3d.ml.torch.ops — hot-path ops backed by libo3dml_amd (HIP, gfx950).

roi_pool (PointRCNN, roipool3d_utils.py:4) and trilinear_devoxelize_* (PVCNN,
pvcnn.py:14) are out of scope: the reference imports them
whenever a GPU is present, so the names exist and a call raises."""
from o3dml_amd.ops import *  # noqa: F401,F403
from o3dml_amd.ops import __all__ as _hot

__all__ = list(_hot) + ["roi_pool", "trilinear_devoxelize_forward", "trilinear_devoxelize_backward"]


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"open3d.ml.torch.ops.{name} is out of scope for o3dml_amd (SURVEY.md §2.2)")
    f.__name__ = name
    return f


roi_pool = _out_of_scope("roi_pool")
trilinear_devoxelize_forward = _out_of_scope("trilinear_devoxelize_forward")
trilinear_devoxelize_backward = _out_of_scope("trilinear_devoxelize_backward")
