"""KPFCNN train step (tests/golden/kpfcnn.npz model + batch): parameter
gradients with the fused BN (csrc/bn.hip) and with torch's modules, each
against the golden; the worst parameters."""
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "tests", "golden"), os.path.join(R, "open3d-ml_amd")]
import test_gpu_kpfcnn as T  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
for flag in ("0", "1"):
    os.environ["O3DML_FUSED_BN"] = flag
    m = T._model(dev)
    m.train(True)
    b = T._ref_batch(dev)
    logits = m(b)
    loss = torch.nn.functional.cross_entropy(logits, b.labels)
    loss.backward()
    res[flag] = ({k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters() if p.grad is not None},
                 logits.detach().cpu().numpy())
    print(flag, "logit err", T._rel(res[flag][1], T.G["train_logits"]), "loss", loss.item(), float(T.G["train_loss"]))
keys = [k[6:] for k in T.G.files if k.startswith("tgrad_")]
rows = []
for k in keys:
    g = T.G["tgrad_" + k]
    rows.append((T._rel(res["1"][0][k], g), T._rel(res["0"][0][k], g), T._rel(res["1"][0][k], res["0"][0][k]), k))
rows.sort(reverse=True)
for r in rows[:25]:
    print("fused %.2e torch %.2e fused-vs-torch %.2e  %s" % r)
