"""open3d.ml: torch ops/layers and contrib backed by o3dml_amd."""
from . import contrib  # noqa: F401
