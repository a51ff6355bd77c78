"""open3d.ml.torch: the hot-path ops and layers (o3dml_amd); importing it also
registers torch.ops.open3d.* as Open3D's op library load does.  models /
pipelines / dataloaders / modules (and configs / datasets / utils / vis) are
Open3D-ML's own, from OPEN3D_ML_ROOT (``open3d._ml3d_alias``)."""
import o3dml_amd as _o3dml

from ... import _ml3d_alias
from . import layers, ops  # noqa: F401

_o3dml.register_torch_ops()


def __getattr__(name):
    return _ml3d_alias.module_getattr(__name__, name)
