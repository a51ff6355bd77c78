"""open3d.ml.torch: the hot-path ops and layers (o3dml_amd); importing it also
registers torch.ops.open3d.* as Open3D's op library load does."""
import o3dml_amd as _o3dml

from . import layers, ops  # noqa: F401

_o3dml.register_torch_ops()
