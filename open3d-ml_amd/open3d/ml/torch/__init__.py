"""open3d.ml.torch: the hot-path ops and layers (o3dml_amd)."""
from . import layers, ops  # noqa: F401
