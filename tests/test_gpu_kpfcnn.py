"""KPFCNN on the GPU vs the reference (tests/golden/kpfcnn.npz: the reference
collate and KPFCNN with oracle-backed Open3D ops, deterministic weights from
randla_weights.fill, S3DIS configuration at first_features_dim 32).

* segmentation_inputs on the GPU (with the rotations the reference drew):
  every layer's points bit-exact, neighbour / pool / upsample matrices
  bit-exact (same canonical neighbour order, same shadow padding and width);
* eval mode and training mode (batch statistics): logits within 1e-4 of the
  logit range, cross-entropy loss within 1e-5 relative, parameter gradients
  within 1e-4 of their range (the reference in fp32 and fp64 agree to ~1e-6,
  so these bounds leave room only for fp32 reduction order and atomics).
Also the HIP max_pool / closest_pool against a torch restatement of
kpconv.py:821-858 with gradients."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import randla_weights  # noqa: E402
from test_kpfcnn import CFG, G  # noqa: E402

pytestmark = pytest.mark.gpu
L = 5


def _model(dev):
    from o3dml_amd.kpfcnn import KPFCNN
    m = KPFCNN(**CFG)
    sd = m.state_dict()
    new = randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd)
    for k in sd:
        if k.endswith("kernel_points"):
            new[k] = torch.from_numpy(G["kp:" + k])
    m.load_state_dict(new)
    return m.to(dev)


def _ref_batch(dev):
    from o3dml_amd.kpfcnn import KPConvBatch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return KPConvBatch([t(G[f"layer_points_{l}"]) for l in range(L)], [t(G[f"neighbors_{l}"]) for l in range(L)],
                       [t(G[f"pools_{l}"]) for l in range(L)], [t(G[f"upsamples_{l}"]) for l in range(L)],
                       [torch.from_numpy(G[f"layer_lengths_{l}"]) for l in range(L)], t(G["features"]),
                       t(G["labels"]).long())


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def test_segmentation_inputs_match_reference(cuda):
    from o3dml_amd.kpfcnn import Config, DEFAULTS, segmentation_inputs
    cfg = Config(DEFAULTS)
    cfg.update(CFG)
    b = segmentation_inputs(cfg, torch.from_numpy(G["points"]).to(cuda), torch.from_numpy(G["features"]).to(cuda),
                            G["labels"], G["lengths"], rotations=list(G["rotations"]))
    for l in range(L):
        assert np.array_equal(b.points[l].cpu().numpy(), G[f"layer_points_{l}"]), f"points layer {l}"
        assert np.array_equal(b.lengths[l].numpy(), G[f"layer_lengths_{l}"]), f"lengths layer {l}"
        for name, got in (("neighbors", b.neighbors), ("pools", b.pools), ("upsamples", b.upsamples)):
            ref = G[f"{name}_{l}"]
            g = got[l].cpu().numpy()
            if ref.shape[0] == 0:
                assert g.shape[0] == 0, f"{name} layer {l}"
                continue
            assert g.shape == ref.shape and np.array_equal(g, ref), f"{name} layer {l}"


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_step_matches_reference(cuda, mode):
    """Logits and loss in both modes, parameter gradients in eval mode at the
    tight bar.  Training-mode gradients (batch statistics) are discontinuous
    in the activations on this fixture — a 1e-7 relative perturbation of
    torch's own BN outputs moves them by ~1e-2 (max-pool argmax ties /
    LeakyReLU kinks, tools/bn_diag3.py) — so they are pinned against that
    rounding envelope by test_step_fused_bn_within_rounding_envelope."""
    m = _model(cuda)
    m.train(mode == "train")
    b = _ref_batch(cuda)
    logits = m(b)
    loss = torch.nn.functional.cross_entropy(logits, b.labels)
    loss.backward()
    assert logits.shape == G[f"{mode}_logits"].shape
    assert _rel(logits.detach().cpu().numpy(), G[f"{mode}_logits"]) < 1e-4
    assert abs(loss.item() - float(G[f"{mode}_loss"])) < 1e-5 * abs(float(G[f"{mode}_loss"]))
    if mode == "train":
        return
    params = dict(m.named_parameters())
    pre = "grad_"
    keys = [k[len(pre):] for k in G.files if k.startswith(pre)]
    assert keys
    for k in keys:
        err = _rel(params[k].grad.cpu().numpy(), G[pre + k])
        assert err < 1e-4, (k, err)


def _train_grads(cuda, bn_act=None):
    from o3dml_amd import kpfcnn
    if bn_act is not None:
        kpfcnn.bn_act = bn_act
        kpfcnn.linear_bn_act = lambda x, w, bn, slope=None: bn_act(torch.nn.functional.linear(x, w), bn, slope)
    m = _model(cuda)
    m.train(True)
    b = _ref_batch(cuda)
    logits = m(b)
    loss = torch.nn.functional.cross_entropy(logits, b.labels)
    loss.backward()
    params = dict(m.named_parameters())
    keys = [k[6:] for k in G.files if k.startswith("tgrad_")]
    return logits, loss, max(_rel(params[k].grad.cpu().numpy(), G["tgrad_" + k]) for k in keys)


def test_step_fused_bn_within_rounding_envelope(cuda, monkeypatch):
    """Training step with the fused BN (csrc/bn.hip): logits and loss at the
    tight bars; the worst parameter-gradient error no larger than twice what
    a 1e-7 relative perturbation of torch's own BN outputs produces on this
    fixture (measured ~1e-2: max-pool argmax / LeakyReLU kinks), i.e. the
    fused BN moves the gradients no more than fp32 rounding of the
    reference's activations does."""
    from o3dml_amd import batchnorm, kpfcnn
    monkeypatch.setattr(kpfcnn, "bn_act", kpfcnn.bn_act)
    monkeypatch.setattr(kpfcnn, "linear_bn_act", kpfcnn.linear_bn_act)
    logits, loss, err = _train_grads(cuda)
    assert _rel(logits.detach().cpu().numpy(), G["train_logits"]) < 1e-4
    assert abs(loss.item() - float(G["train_loss"])) < 1e-5 * abs(float(G["train_loss"]))
    monkeypatch.setenv("O3DML_FUSED_BN", "0")
    env = 0.0
    for sign in (1.0, -1.0):
        gen = torch.Generator(device=cuda).manual_seed(1)

        def noisy(x, bn, slope=None, sign=sign, gen=gen):
            y = batchnorm.bn_act(x, bn, slope)
            return y * (1 + sign * 1e-7 * torch.randn(y.shape, generator=gen, device=y.device))

        env = max(env, _train_grads(cuda, noisy)[2])
    assert env > 1e-4  # the fixture is kink-sensitive (else this test's premise is void)
    assert err <= 2 * env, (err, env)


@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
def test_pooling_matches_torch(cuda, dtype):
    from o3dml_amd.kpfcnn import closest_pool, max_pool
    g = torch.Generator().manual_seed(0)
    ns, n, nb, c = 500, 300, 17, 70
    x = torch.randn((ns, c), generator=g)
    inds = torch.randint(0, ns + 1, (n, nb), generator=g)  # ns = shadow
    inds[:5] = ns
    gout = torch.randn((n, c), generator=g)
    for fn, ref_fn in ((max_pool, lambda xp, i: xp[i].max(1)[0]), (closest_pool, lambda xp, i: xp[i[:, 0]])):
        xr = x.clone().double().requires_grad_(True)
        ref = ref_fn(torch.cat([xr, torch.zeros_like(xr[:1])], 0), inds)
        (ref * gout.double()).sum().backward()
        xg = x.clone().to(cuda).requires_grad_(True)
        out = fn(xg, inds.to(cuda, dtype))
        (out * gout.to(cuda)).sum().backward()
        assert torch.equal(out.detach().cpu().double(), ref.detach())
        assert torch.allclose(xg.grad.cpu().double(), xr.grad, atol=1e-5)
