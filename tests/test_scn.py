"""SparseConvUnet module tree vs the reference (tests/golden/scn.npz, made by
make_golden_scn.py from ml3d/torch/models/sparseconvnet.py): identical
state_dict keys and shapes for the residual and the plain UNet, so reference
checkpoints load unchanged.  The logits are checked on the GPU
(test_gpu_scn.py)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "scn.npz"))


def model(residual):
    from o3dml_amd.sparseconvnet import SparseConvUnet
    return SparseConvUnet(multiplier=8, residual_blocks=residual, conv_block_reps=1, num_classes=5)


@pytest.mark.parametrize("tag,residual", [("res", True), ("plain", False)])
def test_state_dict_manifest(tag, residual):
    sd = model(residual).state_dict()
    assert list(sd.keys()) == [str(k) for k in G[f"{tag}_keys"]]
    assert [",".join(map(str, v.shape)) for v in sd.values()] == [str(s) for s in G[f"{tag}_shapes"]]
