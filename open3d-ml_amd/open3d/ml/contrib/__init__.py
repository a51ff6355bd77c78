"""open3d.ml.contrib: grid subsampling (KPConv) on the GPU.  The box-IoU
helpers Open3D also ships here (imported by the reference's
datasets/utils/operations.py:7 and metrics/__init__.py:5-9, evaluation and
augmentation only) are out of scope: the names exist so
those modules import, a call raises."""
from o3dml_amd.contrib import subsample, subsample_batch  # noqa: F401


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"open3d.ml.contrib.{name} (box IoU for evaluation) is out of scope for "
                                  f"o3dml_amd (SURVEY.md §2.2)")
    f.__name__ = name
    return f


iou_bev_cpu = _out_of_scope("iou_bev_cpu")
iou_3d_cpu = _out_of_scope("iou_3d_cpu")
iou_bev_cuda = _out_of_scope("iou_bev_cuda")
iou_3d_cuda = _out_of_scope("iou_3d_cuda")
