"""The drop-in ``open3d`` namespace exposes every name the reference models
import (SURVEY.md §8b import sites) — CPU only, no compute."""
import importlib

import pytest

IMPORTS = [
    ("open3d.ml.torch.ops", ["voxelize", "ragged_to_dense", "reduce_subarrays_sum", "knn_search",
                             "fixed_radius_search", "build_spatial_hash_table", "furthest_point_sampling",
                             "ball_query", "three_nn", "three_interpolate", "three_interpolate_grad",
                             "nms", "sparse_conv", "sparse_conv_transpose"]),
    ("open3d.ml.torch.layers", ["FixedRadiusSearch", "KNNSearch", "SparseConv", "SparseConvTranspose"]),
    ("open3d.ml.contrib", ["subsample", "subsample_batch"]),
    ("open3d.core", ["Tensor", "nns", "cuda"]),
]


@pytest.mark.parametrize("mod,names", IMPORTS)
def test_reference_import_forms(mod, names):
    m = importlib.import_module(mod)
    for n in names:
        assert hasattr(m, n), f"{mod}.{n}"


def test_build_config_and_nns():
    import open3d
    import open3d.core as o3c
    assert open3d._build_config["BUILD_PYTORCH_OPS"] is True
    assert hasattr(o3c.nns.NearestNeighborSearch, "knn_index")
    assert hasattr(o3c.nns.NearestNeighborSearch, "knn_search")
    assert callable(o3c.cuda.device_count)
    import open3d.ml.torch as ml3d
    assert ml3d.layers.SparseConv is importlib.import_module("o3dml_amd.layers").SparseConv
