"""RandLA-Net module tree vs the reference (tests/golden/randla.npz, generated
by make_golden_randla.py from ml3d/torch/models/randlanet.py): identical
state_dict keys/shapes, and the differentiable (torch) path reproduces the
reference logits on CPU.  The fused HIP path is checked in test_gpu_randla.py."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import randla_weights  # noqa: E402

G = np.load(os.path.join(HERE, "golden", "randla.npz"))


def golden_inputs(to=lambda t: t):
    pc = G["points"]
    inputs = {"features": to(torch.from_numpy(pc)[None])}
    cs, nb, sb, up = [], [], [], []
    cur = pc
    for i in range(4):
        n = G[f"nbr{i}"].astype(np.int64)
        cs.append(to(torch.from_numpy(cur)[None]))
        nb.append(to(torch.from_numpy(n)[None]))
        sb.append(to(torch.from_numpy(n[: cur.shape[0] // 4])[None]))
        up.append(to(torch.from_numpy(G[f"up{i}"].astype(np.int64))[None]))
        cur = cur[: cur.shape[0] // 4]
    inputs.update(coords=cs, neighbor_indices=nb, sub_idx=sb, interp_idx=up)
    return inputs


def golden_model():
    from o3dml_amd.randlanet import RandLANet
    m = RandLANet(num_points=4096)
    sd = m.state_dict()
    m.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()]))
    return m.eval()


def test_state_dict_matches_reference():
    from o3dml_amd.randlanet import RandLANet
    m = RandLANet()
    sd = m.state_dict()
    assert list(sd.keys()) == list(G["keys"])
    assert [",".join(map(str, v.shape)) for v in sd.values()] == list(G["shapes"])
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == int(G["n_params"]) == 1242307


def test_torch_path_matches_reference_logits():
    m = golden_model()
    out = m(golden_inputs())[0].detach().numpy()  # grad enabled -> differentiable torch path
    np.testing.assert_allclose(out, G["logits"], rtol=0, atol=2e-5)
