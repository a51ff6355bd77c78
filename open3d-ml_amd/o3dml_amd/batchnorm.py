"""BatchNorm1d over the point axis + the LeakyReLU after it as two HIP
launches each way (csrc/bn.hip), for KPFCNN's BatchNormBlock / UnaryBlock /
SimpleBlock / ResnetBottleneckBlock (reference ml3d/torch/models/kpconv.py:
1213-1464: ``nn.BatchNorm1d`` on the [1, C, N] view, then ``nn.LeakyReLU``).

``bn_act(x, bn, slope)``: x [N, C] float32 on the GPU, ``bn`` the block's
``nn.BatchNorm1d`` (its weight / bias / running statistics /
num_batches_tracked are used and updated exactly as torch's module does in
train and eval mode), ``slope`` the LeakyReLU slope or None.  Statistics in
double (deterministic block-order sums); the output differs from torch's
fp32 Welford path by fp32 rounding only.

``linear_bn_act(x, weight, bn, slope)``: UnaryBlock's bias-free Linear
folded into the same autograd node (one node instead of the Linear's matmul
+ transpose nodes and the BN's): forward x @ W^T then the BN launches,
backward the BN launches then dX = dZ W and dW = dZ^T x.
"""
import os

import torch

from . import _lib
from ._util import SizeCache, ptr, stream_handle

_WS = SizeCache(lambda n, c: max(int(_lib.load().o3dml_batch_norm_workspace_size(n, c)), 1))


def _ws(n, c, dev):
    return torch.empty(_WS(n, c), dtype=torch.uint8, device=dev)


def _bn_forward(x, weight, bias, bn, training, slope):
    n, c = x.shape
    y = torch.empty_like(x)
    save = torch.empty(4 * c, dtype=torch.float32, device=x.device)
    ws = _ws(n, c, x.device)
    track = training and bn.track_running_stats and bn.running_mean is not None
    if training and bn.momentum is None:
        raise NotImplementedError("bn_act: cumulative moving average (momentum=None)")
    use_running = track or not training
    _lib.call("o3dml_batch_norm_forward", ptr(x), n, c, ptr(weight), ptr(bias),
              ptr(bn.running_mean) if use_running else None, ptr(bn.running_var) if use_running else None,
              ptr(bn.num_batches_tracked) if track else None, float(bn.momentum or 0.0), float(bn.eps),
              int(training), int(slope is not None), float(slope or 0.0), ptr(y), ptr(save), ptr(ws), ws.numel(),
              stream_handle(x.device))
    return y, save


def _bn_backward(g, x, save, training, slope, need_x, need_w, need_b):
    n, c = x.shape
    dx = torch.empty_like(x) if need_x else None
    dw = torch.empty(c, dtype=torch.float32, device=x.device) if need_w else None
    db = torch.empty(c, dtype=torch.float32, device=x.device) if need_b else None
    ws = _ws(n, c, x.device)
    _lib.call("o3dml_batch_norm_backward", ptr(g), ptr(x), n, c, ptr(save), int(training),
              int(slope is not None), float(slope or 0.0), ptr(dx), ptr(dw), ptr(db), ptr(ws), ws.numel(),
              stream_handle(x.device))
    return dx, dw, db


class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, bn, training, slope):
        x = x.contiguous()
        y, save = _bn_forward(x, weight, bias, bn, training, slope)
        ctx.save_for_backward(x, save)
        ctx.meta = (training, slope, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, save = ctx.saved_tensors
        training, slope, has_w, has_b = ctx.meta
        dx, dw, db = _bn_backward(g.contiguous(), x, save, training, slope, ctx.needs_input_grad[0],
                                  has_w and ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2])
        return dx, dw, db, None, None, None


# workspace bytes of the one-call Linear + BN per (n, cin, cout)
_LWS = SizeCache(lambda n, cin, cout: max(int(_lib.load().o3dml_linear_bn_workspace_size(n, cin, cout)), 1))


def _lws(n, cin, cout, dev):
    return torch.empty(_LWS(n, cin, cout), dtype=torch.uint8, device=dev)


class _LinearBnAct(torch.autograd.Function):
    """One C call per direction (csrc/kpfcnn_ops.cpp o3dml_linear_bn_*):
    z = x W^T (rocBLAS), then the BN launches; backward the BN launches then
    dX = dZ W and dW = dZ^T x."""

    @staticmethod
    def forward(ctx, x, w, weight, bias, bn, training, slope):
        x = x.contiguous()
        w_param, w = w, w.detach().contiguous()
        n, cin = x.shape
        cout = w.shape[0]
        z = torch.empty((n, cout), dtype=torch.float32, device=x.device)
        y = torch.empty_like(z)
        save = torch.empty(4 * cout, dtype=torch.float32, device=x.device)
        ws = _lws(n, cin, cout, x.device)
        track = training and bn.track_running_stats and bn.running_mean is not None
        if training and bn.momentum is None:
            raise NotImplementedError("bn_act: cumulative moving average (momentum=None)")
        use_running = track or not training
        _lib.call("o3dml_linear_bn_forward", ptr(x), n, cin, ptr(w), cout, ptr(weight), ptr(bias),
                  ptr(bn.running_mean) if use_running else None, ptr(bn.running_var) if use_running else None,
                  ptr(bn.num_batches_tracked) if track else None, float(bn.momentum or 0.0), float(bn.eps),
                  int(training), int(slope is not None), float(slope or 0.0), ptr(z), ptr(y), ptr(save), ptr(ws),
                  ws.numel(), stream_handle(x.device))
        # the parameter itself (not a detached view): autograd's version check
        # then catches an in-place update between forward and backward
        ctx.save_for_backward(x, w_param, z, save)
        ctx.meta = (training, slope, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, z, save = ctx.saved_tensors
        w = w.detach().contiguous()
        training, slope, has_w, has_b = ctx.meta
        g = g.contiguous()
        n, cin = x.shape
        cout = w.shape[0]
        dev = x.device
        dz = torch.empty((n, cout), dtype=torch.float32, device=dev)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dW = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        dwt = torch.empty(cout, dtype=torch.float32, device=dev) if has_w and ctx.needs_input_grad[2] else None
        db = torch.empty(cout, dtype=torch.float32, device=dev) if has_b and ctx.needs_input_grad[3] else None
        ws = _lws(n, cin, cout, dev)
        _lib.call("o3dml_linear_bn_backward", ptr(g), ptr(x), n, cin, ptr(w), cout, ptr(z), ptr(save), int(training),
                  int(slope is not None), float(slope or 0.0), ptr(dz), ptr(dx), ptr(dW), ptr(dwt), ptr(db), ptr(ws),
                  ws.numel(), stream_handle(dev))
        return dx, dW, dwt, db, None, None, None


def _fused_ok(x, bn):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and isinstance(bn, torch.nn.BatchNorm1d)
            and os.environ.get("O3DML_FUSED_BN", "1") != "0")  # (0: torch's modules, for A/B and debugging)


def bn_act(x, bn, slope=None):
    """LeakyReLU(slope)(bn(x)) (slope None: bn(x)) for x [N, C]; GPU float32
    through csrc/bn.hip, anything else through torch."""
    if not _fused_ok(x, bn):
        y = bn(x)
        return y if slope is None else torch.nn.functional.leaky_relu(y, slope)
    training = bn.training or not bn.track_running_stats
    return _BnAct.apply(x, bn.weight, bn.bias, bn, training, slope)


def linear_bn_act(x, weight, bn, slope=None):
    """bn_act(x @ weight^T, bn, slope) as one autograd node (weight [out, in])."""
    if not _fused_ok(x, bn) or weight.dtype != torch.float32:
        return bn_act(torch.nn.functional.linear(x, weight), bn, slope)
    training = bn.training or not bn.track_running_stats
    return _LinearBnAct.apply(x, weight, bn.weight, bn.bias, bn, training, slope)
