"""open3d.ml.torch.ops — hot-path ops backed by libo3dml_amd (HIP, gfx950)."""
from o3dml_amd.ops import *  # noqa: F401,F403
from o3dml_amd.ops import __all__  # noqa: F401
