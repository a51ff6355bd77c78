"""open3d.ml.contrib: grid subsampling (KPConv) on the GPU."""
from o3dml_amd.contrib import subsample, subsample_batch  # noqa: F401
