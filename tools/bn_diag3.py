"""Sensitivity of the KPFCNN train-step gradients (golden model) to 1-ulp
scale perturbations of the BN outputs, torch's BN throughout: if relative
noise of 1e-7 on activations moves encoder_blocks.{0,2} gradients by ~1e-3
(max-pool argmax / LeakyReLU kinks), the golden's 1e-4 bar on them measures
agreement with torch's exact rounding, not correctness."""
import os
import sys

import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "tests", "golden"), os.path.join(R, "open3d-ml_amd")]
os.environ["O3DML_FUSED_BN"] = "0"
import test_gpu_kpfcnn as T  # noqa: E402
from o3dml_amd import batchnorm, kpfcnn  # noqa: E402

dev = torch.device("cuda", 0)
orig = batchnorm.bn_act
for eps in (0.0, 1e-7, -1e-7, 3e-7):
    g = torch.Generator(device=dev).manual_seed(1)

    def noisy(x, bn, slope=None):
        y = orig(x, bn, slope)
        if eps:
            y = y * (1 + eps * torch.randn(y.shape, generator=g, device=dev))
        return y

    kpfcnn.bn_act = noisy
    m = T._model(dev)
    m.train(True)
    b = T._ref_batch(dev)
    logits = m(b)
    torch.nn.functional.cross_entropy(logits, b.labels).backward()
    params = dict(m.named_parameters())
    keys = [k[6:] for k in T.G.files if k.startswith("tgrad_")]
    errs = sorted(((T._rel(params[k].grad.cpu().numpy(), T.G["tgrad_" + k]), k) for k in keys), reverse=True)
    print(f"eps {eps:+.0e}: logits {T._rel(logits.detach().cpu().numpy(), T.G['train_logits']):.1e} worst", 
          ", ".join(f"{k} {e:.2e}" for e, k in errs[:3]), flush=True)
