"""Per-BN check inside the KPFCNN train step: every bn_act call also runs
torch's BatchNorm1d (+ LeakyReLU) on a copy of the module and input; on the
backward, the fused kernel's (dx, dw, db) for the incoming gradient vs torch's
autograd.grad of the copy."""
import copy
import os
import sys

import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "tests", "golden"), os.path.join(R, "open3d-ml_amd")]
import test_gpu_kpfcnn as T  # noqa: E402
from o3dml_amd import batchnorm, kpfcnn  # noqa: E402

dev = torch.device("cuda", 0)
orig = batchnorm.bn_act
calls = []


def rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def spy(x, bn, slope=None):
    bt = copy.deepcopy(bn)
    xt = x.detach().clone().requires_grad_()
    yt = bt(xt)
    if slope is not None:
        yt = torch.nn.functional.leaky_relu(yt, slope)
    y = orig(x, bn, slope)
    i = len(calls)
    calls.append((x.shape, slope))


    def hook(g):
        gx, gw, gb = torch.autograd.grad(yt, (xt, bt.weight, bt.bias), g, retain_graph=True)
        # fused backward of the same g (a second identical forward keeps save)
        x2 = x.detach().clone().requires_grad_()
        bn2 = copy.deepcopy(bn)
        for p in bn2.parameters():
            p.grad = None
        bn2.train(bn.training)
        bn2.running_mean.copy_(bt.running_mean)  # irrelevant to grads
        with torch.enable_grad():
            y2 = orig(x2, bn2, slope)
            y2.backward(g)
        print(f"  bn{i} bwd: dx {rel(x2.grad, gx):.2e} dw {rel(bn2.weight.grad, gw):.2e} db {rel(bn2.bias.grad, gb):.2e}"
              f" |g| {float(g.abs().max()):.3e} zeros {float((g == 0).float().mean()):.3f}", flush=True)
    y.register_hook(hook)
    return y


kpfcnn.bn_act = spy
m = T._model(dev)
m.train(True)
b = T._ref_batch(dev)
logits = m(b)
torch.nn.functional.cross_entropy(logits, b.labels).backward()
