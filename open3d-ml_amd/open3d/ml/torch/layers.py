"""open3d.ml.torch.layers — FixedRadiusSearch, KNNSearch, SparseConv, SparseConvTranspose."""
from o3dml_amd.layers import FixedRadiusSearch, KNNSearch, SparseConv, SparseConvTranspose  # noqa: F401
