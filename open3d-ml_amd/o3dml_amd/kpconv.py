"""KPConv on MI355X (reference ml3d/torch/models/kpconv.py
KPConv class, :893-1159).

``KPConv`` keeps the reference parameters (``weights`` [K, Cin, Cout],
``kernel_points`` [K, 3] non-trainable, and for deformable convolutions
``offset_conv`` / ``offset_bias``) so reference state_dicts load unchanged.
Forward = fused neighbourhood aggregation in HIP (csrc/kpconv.hip:
influences of every (neighbour, kernel point) + weighted feature sums, with
shadow neighbours skipped) followed by one dense GEMM
[n, K*Cin] @ [K*Cin, Cout].  Gradients flow to the features and the weights
(feature gradient by the fused backward kernel with fp32 atomics); the
shared kernel-point positions are constants, as in the reference
(requires_grad False); deformable convolutions train end to end: the HIP
kernel-point / modulation gradient (o3dml_kpconv_kernel_point_grad) flows
into the offset convolution, and min_d2 feeds p2p_fitting_regularizer.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from ._util import SizeCache, gpu_device, index_bits, ptr, stream_handle, to_dev, workspace

_INFLUENCE = {"constant": 0, "linear": 1, "gaussian": 2}


def _wf_forward(x, q_pts, s_pts, nbr, kp, kp_per_query, extent, influence, closest, mod):
    n, nb = nbr.shape
    K = kp.shape[-2]
    cin = x.shape[1]
    out = torch.empty((n, K, cin), dtype=torch.float32, device=x.device)
    _lib.call("o3dml_kpconv_weighted_features", ptr(q_pts), n, ptr(s_pts), s_pts.shape[0], ptr(nbr),
              index_bits(nbr.dtype), nb, ptr(x), cin, ptr(kp), K, int(kp_per_query), float(extent), influence,
              int(closest), ptr(mod), ptr(out), stream_handle(x.device))
    return out


def _wf_backward_x(gm, q_pts, s_pts, nbr, kp, kp_per_query, extent, influence, closest, n_s, cin):
    """dX of the aggregation for dWF gm (modulations already folded in)."""
    n, nb = nbr.shape
    K = kp.shape[-2]
    if torch.are_deterministic_algorithms_enabled():
        # fixed-order gather over the inverse neighbour lists (no fp32 atomics)
        dx = torch.empty((n_s, cin), dtype=torch.float32, device=gm.device)
        ws = workspace(_lib.load().o3dml_kpconv_inverse_workspace_size(n, nb, n_s), gm.device)
        _lib.call("o3dml_kpconv_weighted_features_backward_det", ptr(q_pts), n, ptr(s_pts), n_s, ptr(nbr),
                  index_bits(nbr.dtype), nb, ptr(gm), cin, ptr(kp), K, int(kp_per_query), float(extent),
                  influence, int(closest), ptr(dx), ptr(ws), ws.numel(), stream_handle(gm.device))
    else:
        dx = torch.zeros((n_s, cin), dtype=torch.float32, device=gm.device)
        _lib.call("o3dml_kpconv_weighted_features_backward", ptr(q_pts), n, ptr(s_pts), n_s, ptr(nbr),
                  index_bits(nbr.dtype), nb, ptr(gm), cin, ptr(kp), K, int(kp_per_query), float(extent),
                  influence, int(closest), ptr(dx), stream_handle(gm.device))
    return dx


class _WeightedFeatures(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, q_pts, s_pts, nbr, kp, kp_per_query, extent, influence, closest, modulations):
        kpd = kp.detach().contiguous()
        mod = None if modulations is None else modulations.detach().contiguous()
        out = _wf_forward(x, q_pts, s_pts, nbr, kpd, kp_per_query, extent, influence, closest, mod)
        ctx.save_for_backward(x, q_pts, s_pts, nbr, kpd, mod if mod is not None else torch.empty(0, device=x.device))
        ctx.meta = (kp_per_query, extent, influence, closest, x.shape[0], x.shape[1], mod is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        x, q_pts, s_pts, nbr, kp, mod = ctx.saved_tensors
        kp_per_query, extent, influence, closest, n_s, cin, has_mod = ctx.meta
        n, nb = nbr.shape
        K = kp.shape[-2]
        g = g.contiguous()
        dx = dkp = dmod = None
        if ctx.needs_input_grad[0]:
            gm = g * mod[:, :, None] if has_mod else g  # the modulation scales dWF (kpconv.py:1149-1150)
            dx = _wf_backward_x(gm.contiguous(), q_pts, s_pts, nbr, kp, kp_per_query, extent, influence, closest,
                                n_s, cin)
        if ctx.needs_input_grad[4] or (has_mod and ctx.needs_input_grad[9]):
            if not kp_per_query:
                raise NotImplementedError("KPConv: gradients w.r.t. shared (non-deformed) kernel points")
            dkp = torch.empty((n, K, 3), dtype=torch.float32, device=g.device)
            dm = torch.empty((n, K), dtype=torch.float32, device=g.device) if has_mod else None
            _lib.call("o3dml_kpconv_kernel_point_grad", ptr(q_pts), n, ptr(s_pts), s_pts.shape[0], ptr(nbr),
                      index_bits(nbr.dtype), nb, ptr(x), cin, ptr(g), ptr(kp), K, float(extent), influence,
                      int(closest), ptr(mod) if has_mod else None, ptr(dkp), ptr(dm), stream_handle(g.device))
            dmod = dm
        return dx, None, None, None, dkp, None, None, None, None, dmod


# (n, nb, n_support, K, cin, cout, deterministic) -> workspace bytes
_KWS = SizeCache(lambda *key: max(int(_lib.load().o3dml_kpconv_rigid_workspace_size(*key)), 1))


class _KPConvRigid(torch.autograd.Function):
    """Rigid KPConv as ONE autograd node and one C call per direction
    (csrc/kpfcnn_ops.cpp o3dml_kpconv_rigid_*): the HIP aggregation WF [n, K,
    Cin] and out = WF.view(n, K Cin) @ W.view(K Cin, Cout) (rocBLAS) forward;
    dW = WF^T g, dWF = g W^T and the aggregation backward backward."""

    @staticmethod
    def _ws(n, nb, ns, K, cin, cout, det, dev):
        return torch.empty(_KWS(n, nb, ns, K, cin, cout, det), dtype=torch.uint8, device=dev)

    @staticmethod
    def forward(ctx, x, w, q_pts, s_pts, nbr, kp, extent, influence, closest):
        kpd = kp.detach().contiguous()
        w2 = w.detach().reshape(-1, w.shape[-1]).contiguous()
        n, nb = nbr.shape
        K, cin, cout = kpd.shape[-2], x.shape[1], w2.shape[1]
        wf = torch.empty((n, K, cin), dtype=torch.float32, device=x.device)
        out = torch.empty((n, cout), dtype=torch.float32, device=x.device)
        ws = _KPConvRigid._ws(n, nb, s_pts.shape[0], K, cin, cout, 0, x.device)
        _lib.call("o3dml_kpconv_rigid_forward", ptr(q_pts), n, ptr(s_pts), s_pts.shape[0], ptr(nbr),
                  index_bits(nbr.dtype), nb, ptr(x), cin, ptr(kpd), K, float(extent), influence, int(closest),
                  ptr(w2), cout, ptr(wf), ptr(out), ptr(ws), ws.numel(), stream_handle(x.device))
        # the parameter itself (not a detached view): autograd's version check
        # then catches an in-place update between forward and backward
        ctx.save_for_backward(w, wf, q_pts, s_pts, nbr, kpd)
        ctx.meta = (extent, influence, closest, x.shape[0], tuple(w.shape))
        return out

    @staticmethod
    def backward(ctx, g):
        w, wf, q_pts, s_pts, nbr, kp = ctx.saved_tensors
        w2 = w.detach().reshape(-1, w.shape[-1]).contiguous()
        extent, influence, closest, n_s, wshape = ctx.meta
        n, K, cin = wf.shape
        nb = nbr.shape[1]
        cout = w2.shape[1]
        dev = wf.device
        g = g.contiguous()
        dw = torch.empty(wshape, dtype=torch.float32, device=dev) if ctx.needs_input_grad[1] else None
        need_x = ctx.needs_input_grad[0]
        det = int(need_x and torch.are_deterministic_algorithms_enabled())
        dx = torch.empty((n_s, cin), dtype=torch.float32, device=dev) if need_x else None
        gwf = torch.empty((n, K * cin), dtype=torch.float32, device=dev) if need_x else None
        ws = _KPConvRigid._ws(n, nb, n_s, K, cin, cout, det, dev)
        _lib.call("o3dml_kpconv_rigid_backward", ptr(q_pts), n, ptr(s_pts), n_s, ptr(nbr), index_bits(nbr.dtype), nb,
                  ptr(g), cin, ptr(kp), K, float(extent), influence, int(closest), ptr(w2), cout, ptr(wf), ptr(gwf),
                  ptr(dx), ptr(dw), det, ptr(ws), ws.numel(), stream_handle(dev))
        return dx, dw, None, None, None, None, None, None, None


def min_d2(q_pts, s_pts, neighb_inds, kernel_points):
    """The deformable reference's min_d2 [n, K] (kpconv.py:1071): squared
    distance from each (deformed) kernel point to its nearest neighbour, the
    shadow neighbour at 1e6 included.  The nearest column comes from the HIP
    kernel; the distance is recomputed with torch ops so p2p_fitting_regularizer
    differentiates into the kernel points (kpconv.py:2167-2209)."""
    dev = kernel_points.device
    nbr = neighb_inds if neighb_inds.dtype in (torch.int32, torch.int64) else neighb_inds.long()
    n, nb = nbr.shape
    K = kernel_points.shape[-2]
    col = torch.empty((n, K), dtype=torch.int32, device=dev)
    # operands bound to names: a temporary freed inside the argument list could
    # be handed to the next temporary by the caching allocator before the launch
    nbr_c, kp_c = nbr.contiguous(), kernel_points.detach().contiguous()
    _lib.call("o3dml_kpconv_min_d2_columns", ptr(q_pts), n, ptr(s_pts), s_pts.shape[0], ptr(nbr_c),
              index_bits(nbr.dtype), nb, ptr(kp_c), K, ptr(col),
              stream_handle(dev))
    s_ext = torch.cat((s_pts, torch.zeros_like(s_pts[:1, :]) + 1e6), 0)
    ids = torch.gather(nbr.long(), 1, col.long()).clamp_(0, s_pts.shape[0])
    nbp = s_ext[ids] - q_pts.unsqueeze(1)  # [n, K, 3]
    return torch.sum((nbp - kernel_points) ** 2, dim=2)


def weighted_features(q_pts, s_pts, neighb_inds, x, kernel_points, extent, influence="linear",
                      aggregation_mode="sum", modulations=None):
    """WF[n, k, :] = sum_j influence(|s_j - q_n - kp_k|) * x[j] over the neighbours
    of q_n (shadow index = len(s_pts) contributes zero): kpconv.py:1046-1145.
    kernel_points [K, 3] or per-query [n, K, 3] (deformable: differentiable,
    out-of-range neighbours dropped as the reference's filter does);
    modulations [n, K] or None (differentiable)."""
    dev = gpu_device(x)
    if influence not in _INFLUENCE:
        raise ValueError("Unknown influence function type (config.KP_influence)")
    if aggregation_mode not in ("sum", "closest"):
        raise ValueError("Unknown convolution mode. Should be 'closest' or 'sum'")
    if kernel_points.requires_grad and kernel_points.dim() != 3:
        raise NotImplementedError("KPConv: gradients w.r.t. shared (non-deformed) kernel points are not supported")
    qp = to_dev(q_pts, dev, torch.float32)
    sp = to_dev(s_pts, dev, torch.float32)
    nbr = to_dev(neighb_inds, dev)
    if nbr.dtype not in (torch.int32, torch.int64):
        nbr = nbr.long()
    kp = kernel_points.to(dev).float()
    mod = None if modulations is None else modulations.to(dev).float()
    xx = x if x.is_cuda else x.to(dev)
    return _WeightedFeatures.apply(xx.float().contiguous(), qp, sp, nbr.contiguous(), kp, kp.dim() == 3,
                                   float(extent), _INFLUENCE[influence], aggregation_mode == "closest", mod)


def kpconv_rigid(q_pts, s_pts, neighb_inds, x, kernel_points, weights, extent, influence="linear",
                 aggregation_mode="sum"):
    """KPConv.forward for rigid kernel points: sum_k WF[:, k] @ W[k] with WF
    the weighted neighbour features (kpconv.py:1046-1159), one autograd node
    (_KPConvRigid)."""
    dev = gpu_device(x)
    if influence not in _INFLUENCE:
        raise ValueError("Unknown influence function type (config.KP_influence)")
    if aggregation_mode not in ("sum", "closest"):
        raise ValueError("Unknown convolution mode. Should be 'closest' or 'sum'")
    if kernel_points.requires_grad:
        raise NotImplementedError("KPConv: gradients w.r.t. shared (non-deformed) kernel points are not supported")
    qp = to_dev(q_pts, dev, torch.float32)
    sp = to_dev(s_pts, dev, torch.float32)
    nbr = to_dev(neighb_inds, dev)
    if nbr.dtype not in (torch.int32, torch.int64):
        nbr = nbr.long()
    kp = kernel_points if kernel_points.is_cuda and kernel_points.dtype == torch.float32 else \
        kernel_points.to(dev).float()
    xx = x if x.is_cuda else x.to(dev)
    return _KPConvRigid.apply(xx.float().contiguous(), weights, qp, sp, nbr.contiguous(), kp, float(extent),
                              _INFLUENCE[influence], aggregation_mode == "closest")


def _sphere_points(radius, K, fixed):
    """Deterministic kernel disposition (Fibonacci sphere at 2/3 radius, centre
    point first when fixed='center').  The reference optimises its dispositions
    (kernels/kernel_points.py); trained checkpoints carry theirs in the
    state_dict ``kernel_points`` entry, which this module loads unchanged."""
    pts = []
    m = K - 1 if fixed == "center" else K
    if fixed == "center":
        pts.append([0.0, 0.0, 0.0])
    ga = math.pi * (3.0 - math.sqrt(5.0))
    for i in range(m):
        z = 1 - 2 * (i + 0.5) / max(m, 1)
        r = math.sqrt(max(0.0, 1 - z * z))
        pts.append([r * math.cos(ga * i), r * math.sin(ga * i), z])
    return np.asarray(pts, np.float32) * (radius * 2.0 / 3.0)


class KPConv(nn.Module):
    """Reference-compatible KPConv (kpconv.py:893-1159)."""

    def __init__(self, kernel_size, p_dim, in_channels, out_channels, KP_extent, radius,
                 fixed_kernel_points="center", KP_influence="linear", aggregation_mode="sum", deformable=False,
                 modulated=False):
        super().__init__()
        self.K = kernel_size
        self.p_dim = p_dim
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.radius = radius
        self.KP_extent = KP_extent
        self.fixed_kernel_points = fixed_kernel_points
        self.KP_influence = KP_influence
        self.aggregation_mode = aggregation_mode
        self.deformable = deformable
        self.modulated = modulated
        self.min_d2 = None
        self.deformed_KP = None
        self.offset_features = None
        self.weights = nn.Parameter(torch.zeros((self.K, in_channels, out_channels), dtype=torch.float32))
        if deformable:
            self.offset_dim = (p_dim + 1) * self.K if modulated else p_dim * self.K
            self.offset_conv = KPConv(self.K, p_dim, in_channels, self.offset_dim, KP_extent, radius,
                                      fixed_kernel_points=fixed_kernel_points, KP_influence=KP_influence,
                                      aggregation_mode=aggregation_mode)
            self.offset_bias = nn.Parameter(torch.zeros(self.offset_dim, dtype=torch.float32))
        else:
            self.offset_dim = None
            self.offset_conv = None
            self.offset_bias = None
        nn.init.kaiming_uniform_(self.weights, a=math.sqrt(5))
        if deformable:
            self.kernel_points = self.offset_conv.kernel_points
        else:
            self.kernel_points = nn.Parameter(torch.from_numpy(_sphere_points(radius, self.K, fixed_kernel_points)),
                                              requires_grad=False)

    def forward(self, q_pts, s_pts, neighb_inds, x):
        modulations = None
        kp = self.kernel_points
        if self.deformable:
            self.offset_features = self.offset_conv(q_pts, s_pts, neighb_inds, x) + self.offset_bias
            if self.modulated:
                unscaled = self.offset_features[:, :self.p_dim * self.K].view(-1, self.K, self.p_dim)
                modulations = 2 * torch.sigmoid(self.offset_features[:, self.p_dim * self.K:])
            else:
                unscaled = self.offset_features.view(-1, self.K, self.p_dim)
            self.deformed_KP = unscaled * self.KP_extent + self.kernel_points
            kp = self.deformed_KP
            # distances kept for p2p_fitting_regularizer (kpconv.py:1071)
            self.min_d2 = min_d2(q_pts, s_pts, neighb_inds, kp)
        if not self.deformable and self.weights.dtype == torch.float32:
            return kpconv_rigid(q_pts, s_pts, neighb_inds, x, kp, self.weights, self.KP_extent, self.KP_influence,
                                self.aggregation_mode)
        wf = weighted_features(q_pts, s_pts, neighb_inds, x, kp, self.KP_extent, self.KP_influence,
                               self.aggregation_mode, modulations)
        n = wf.shape[0]
        return wf.reshape(n, -1) @ self.weights.reshape(-1, self.out_channels)
