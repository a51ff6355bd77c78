"""open3d.core subset: Tensor (numpy/torch interop), nns, cuda.device_count."""
from o3dml_amd.core import Device, Dtype, Tensor, cuda, nns  # noqa: F401
