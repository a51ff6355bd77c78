"""open3d.ml: torch ops/layers and contrib backed by o3dml_amd; configs /
datasets / utils / vis are Open3D-ML's own (``open3d._ml3d_alias``)."""
from .. import _ml3d_alias
from . import contrib  # noqa: F401


def __getattr__(name):
    return _ml3d_alias.module_getattr(__name__, name)
