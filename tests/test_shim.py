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


# --- open3d.ml namespace from OPEN3D_ML_ROOT (upstream open3d/ml/torch/__init__.py;
# the reference's set_open3d_ml_root.sh:3, docs/howtos.md:235-245, tests/test_models.py:36-38)
_FAKE_ML3D = {
    "ml3d/__init__.py": "",
    "ml3d/torch/__init__.py": "",
    "ml3d/torch/models/__init__.py": (
        "from open3d.ml.torch.ops import knn_search\n"
        "from open3d.ml.torch.layers import FixedRadiusSearch\n"
        "from open3d.ml.contrib import subsample\n"
        "import open3d.core as o3c\n"
        "class RandLANet:\n"
        "    bound = (knn_search, FixedRadiusSearch, subsample, o3c.nns.NearestNeighborSearch)\n"
        "    def __init__(self, **kw):\n"
        "        self.cfg = kw\n"),
    "ml3d/torch/models/extra.py": "from . import RandLANet\nclass Extra(RandLANet):\n    pass\n",
    "ml3d/torch/pipelines/__init__.py": "class SemanticSegmentation:\n    pass\n",
    "ml3d/torch/dataloaders/__init__.py": "class TorchDataloader:\n    pass\n",
    "ml3d/torch/modules/__init__.py": "class SemSegLoss:\n    pass\n",
    "ml3d/datasets/__init__.py": "class SemanticKITTI:\n    pass\n",
    "ml3d/utils/__init__.py": "MODEL = {}\n",
    "ml3d/configs/__init__.py": "",
    "ml3d/vis/__init__.py": "import open3d.visualization.gui  # the GUI: never imported unless used\n",
}

_CHECK_WITH_ROOT = r"""
import sys
import open3d
import open3d.ml.torch as ml3d
import o3dml_amd
assert open3d._build_config["BUNDLE_OPEN3D_ML"] is True
net = ml3d.models.RandLANet(num_points=5000, num_classes=10, in_channels=6)
assert net.cfg["num_points"] == 5000
assert type(net).__module__ == "ml3d.torch.models"
knn, frs, sub, nns = type(net).bound
assert knn is o3dml_amd.ops.knn_search and frs is o3dml_amd.layers.FixedRadiusSearch
assert sub is o3dml_amd.contrib.subsample and nns is o3dml_amd.core.nns.NearestNeighborSearch
from open3d.ml.torch.models import RandLANet
assert RandLANet is ml3d.models.RandLANet
import open3d.ml.torch.pipelines as P
assert P is sys.modules["ml3d.torch.pipelines"] and ml3d.pipelines.SemanticSegmentation
assert ml3d.dataloaders.TorchDataloader and ml3d.modules.SemSegLoss
assert open3d.ml.datasets.SemanticKITTI is ml3d.datasets.SemanticKITTI
assert open3d.ml.utils.MODEL == {} and open3d.ml.configs
assert ml3d.ops.knn_search is o3dml_amd.ops.knn_search and ml3d.layers.SparseConv is o3dml_amd.layers.SparseConv
assert "ml3d.vis" not in sys.modules
# a submodule below an aliased package is the ml3d module itself (one copy,
# one class object), and aliased modules keep their own spec
import open3d.ml.torch.models.extra as E
from open3d.ml.torch.models.extra import Extra
assert E is sys.modules["ml3d.torch.models.extra"] and Extra is E.Extra
assert issubclass(Extra, ml3d.models.RandLANet)
for name in ("ml3d.torch.models", "ml3d.torch.pipelines", "ml3d.torch.models.extra"):
    sp = sys.modules[name].__spec__
    assert sp.name == name and sp.origin and sp.origin.endswith(".py"), (name, sp)
assert list(sys.modules["ml3d.torch.models"].__spec__.submodule_search_locations)
print("NAMESPACE OK")
"""

_CHECK_WITHOUT_ROOT = r"""
import open3d
import open3d.ml.torch as ml3d
assert open3d._build_config["BUNDLE_OPEN3D_ML"] is False
assert not hasattr(ml3d, "models") and not hasattr(open3d.ml, "datasets")
try:
    ml3d.pipelines
except AttributeError as e:
    assert "OPEN3D_ML_ROOT" in str(e)
try:
    import open3d.ml.torch.models
    raise SystemExit("imported without a checkout")
except ModuleNotFoundError:
    pass
assert ml3d.ops.knn_search
print("NAMESPACE OK")
"""


def _run_py(code, env_extra, cwd):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("OPEN3D_ML_ROOT", "PYTHONPATH")}
    env["PYTHONPATH"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "open3d-ml_amd")
    env.update(env_extra)
    return subprocess.run([sys.executable, "-c", code], env=env, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_open3d_ml_root_routes_models_to_checkout(tmp_path):
    """`import open3d.ml.torch as ml3d; ml3d.models.X` resolves to the
    OPEN3D_ML_ROOT checkout's ml3d (a tiny fake tree here: no reference code
    travels), whose own op imports land on this build's ops."""
    root = tmp_path / "Open3D-ML"
    for rel, text in _FAKE_ML3D.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    r = _run_py(_CHECK_WITH_ROOT, {"OPEN3D_ML_ROOT": str(root)}, str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert f"Using external Open3D-ML in {root}" in r.stdout
    assert "NAMESPACE OK" in r.stdout


def test_open3d_ml_without_checkout_says_so(tmp_path):
    r = _run_py(_CHECK_WITHOUT_ROOT, {}, str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "NAMESPACE OK" in r.stdout


_CHECK_REFERENCE = r"""
import sys, types
# third-party modules absent from the image (SURVEY.md §0.3): addict, tensorboard
class Dict(dict):
    def __getattr__(s, k):
        try:
            return s[k]
        except KeyError:
            raise AttributeError(k)
    def __setattr__(s, k, v):
        s[k] = v
sys.modules["addict"] = types.SimpleNamespace(Dict=Dict)
tb = types.ModuleType("torch.utils.tensorboard"); tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = tb
import open3d.ml.torch as ml3d
import o3dml_amd
from o3dml_amd import kpfcnn, randlanet, sparseconvnet
import ml3d.torch.models.kpconv as K, ml3d.torch.models.sparseconvnet as S, ml3d.datasets.utils.dataprocessing as D
assert K.FixedRadiusSearch is o3dml_amd.layers.FixedRadiusSearch and K.ragged_to_dense is o3dml_amd.ops.ragged_to_dense
assert S.SparseConv is o3dml_amd.layers.SparseConv and S.voxelize is o3dml_amd.ops.voxelize
assert D.subsample is o3dml_amd.contrib.subsample
man = lambda m: {k: tuple(v.shape) for k, v in m.state_dict().items()}
pairs = [(ml3d.models.RandLANet(num_points=45056, num_classes=19), randlanet.RandLANet(num_points=45056, num_classes=19)),
         (ml3d.models.SparseConvUnet(), sparseconvnet.SparseConvUnet()), (ml3d.models.KPFCNN(), kpfcnn.KPFCNN())]
for a, b in pairs:
    assert type(a).__module__.startswith("ml3d.torch.models"), type(a)
    assert man(a) == man(b), type(a).__name__
assert ml3d.models.PointPillars and ml3d.models.PointTransformer and ml3d.pipelines.SemanticSegmentation
print("REFERENCE NAMESPACE OK")
"""


@pytest.mark.skipif(not __import__("os").path.isdir("/root/reference/ml3d"),
                    reason="the reference checkout exists only in the build container")
def test_reference_checkout_through_namespace(tmp_path):
    """OPEN3D_ML_ROOT=<the reference checkout>: its model zoo imports through
    this shim (its op imports bound to o3dml_amd), and RandLANet /
    SparseConvUnet / KPFCNN built from it have this build's state_dict
    layout, key for key and shape for shape (construction only, no compute)."""
    r = _run_py(_CHECK_REFERENCE, {"OPEN3D_ML_ROOT": "/root/reference"}, str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "REFERENCE NAMESPACE OK" in r.stdout
