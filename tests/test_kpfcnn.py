"""KPFCNN module tree and collate plumbing vs the reference (tests/golden/
kpfcnn.npz, made by make_golden_kpfcnn.py from ml3d/torch/models/kpconv.py and
ml3d/torch/dataloaders/concat_batcher.py): identical state_dict keys and
shapes (reference checkpoints load unchanged) and the random grid rotations
drawn from a seeded np.random (kpconv.py:2063-2080).  The collate and the
logits are checked on the GPU (test_gpu_kpfcnn.py)."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "kpfcnn.npz"))
CFG = dict(lbl_values=list(range(13)), num_classes=13, ignored_label_inds=[], first_subsampling_dl=0.04,
           in_features_dim=5, first_features_dim=32, batch_norm_momentum=0.98, conv_radius=2.5,
           KP_extent=1.2, num_kernel_points=15)


def test_state_dict_manifest():
    from o3dml_amd.kpfcnn import KPFCNN
    sd = KPFCNN(**CFG).state_dict()
    assert list(sd.keys()) == [str(k) for k in G["keys"]]
    assert [",".join(map(str, v.shape)) for v in sd.values()] == [str(s) for s in G["shapes"]]


def test_random_rotations_follow_reference_draws():
    """Same np.random consumption as batch_grid_subsampling: after seed(0) the
    four subsampling calls draw the reference's rotations (fp32 rounding of the
    Rodrigues terms may differ by an ulp)."""
    from o3dml_amd.kpfcnn import random_rotations
    np.random.seed(0)
    B = len(G["lengths"])
    ours = np.stack([random_rotations(B) for _ in range(len(G["rotations"]))])
    assert np.abs(ours - G["rotations"]).max() < 1e-6
    # proper rotations
    for R in ours.reshape(-1, 3, 3):
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-6) and abs(np.linalg.det(R) - 1) < 1e-5
