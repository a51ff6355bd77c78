"""open3d.ml.torch.layers — FixedRadiusSearch, RadiusSearch, KNNSearch, SparseConv, SparseConvTranspose."""
from o3dml_amd.layers import FixedRadiusSearch, KNNSearch, RadiusSearch, SparseConv, SparseConvTranspose  # noqa: F401
