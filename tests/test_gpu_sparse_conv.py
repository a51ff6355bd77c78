"""GPU parity for sparse convolution: rulebook (Linf
neighbours + kernel index) bit-exact vs the oracle; features vs the oracle's
double-accumulated conv within rtol 1e-4 (BASELINE north_star tolerance);
gradients vs float64 torch autograd of the same CSR convolution, rtol 1e-4."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def _voxels(n, extent, seed):
    rng = np.random.default_rng(seed)
    v = np.unique(rng.integers(0, extent, (n, 3)), axis=0)
    return (v + 0.5).astype(np.float32)


def _csr_conv64(W, x, nidx, kidx, rs, bias=None):
    """float64 torch reference: out[o] = sum_pairs x[idx] @ W[kidx]."""
    K = int(np.prod(W.shape[:-2]))
    Wf = W.reshape(K, W.shape[-2], W.shape[-1])
    n_out = rs.shape[0] - 1
    o = torch.repeat_interleave(torch.arange(n_out), rs[1:] - rs[:-1])
    contrib = torch.einsum("pc,pcd->pd", x[nidx.long()], Wf[kidx.long()])
    out = torch.zeros((n_out, W.shape[-1]), dtype=torch.float64).index_add_(0, o, contrib)
    return out if bias is None else out + bias


def _close_elem(a, b, s, rtol=RTOL, floor=1e-6):
    """Per element against the float64 truth b: |a - b| <= rtol |b| + floor * s,
    s = the element's sum of |term| (sum over its pairs of |x| . |W|): the
    absolute floor only matters where the terms cancel (|b| << s); 1e-6 s is
    ~16 units of fp32 roundoff of the summed magnitudes."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    s = np.asarray(s, np.float64)
    err = np.abs(a - b)
    bound = rtol * np.abs(b) + floor * s
    assert (err <= bound).all(), f"worst err / bound {float((err / bound).max()):.3e}, max rel {float((err / np.maximum(np.abs(b), 1e-300)).max()):.3e}"


def _truth64(W, x, nidx, kidx, rs, bias=None):
    """(float64 output, per-element term magnitude sum) of the CSR conv."""
    W = torch.as_tensor(np.asarray(W), dtype=torch.float64)
    x = torch.as_tensor(np.asarray(x), dtype=torch.float64)
    nidx, kidx, rs = (torch.as_tensor(np.asarray(t)) for t in (nidx, kidx, rs))
    out = _csr_conv64(W, x, nidx, kidx, rs, None if bias is None else torch.as_tensor(np.asarray(bias), dtype=torch.float64))
    mag = _csr_conv64(W.abs(), x.abs(), nidx, kidx, rs)
    if bias is not None:
        mag = mag + torch.as_tensor(np.abs(np.asarray(bias)), dtype=torch.float64)
    return out.numpy(), mag.numpy()


def _close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.abs(b).max() + 1e-12
    assert np.abs(a - b).max() <= rtol * scale, f"max err {np.abs(a - b).max() / scale:.3e} (rel to max)"


@pytest.mark.parametrize("cin,cout", [(32, 32), (3, 16), (64, 96), (96, 224), (64, 128), (1, 32), (2, 16),
                                      (4, 64), (3, 24)])
def test_submanifold_conv_forward(cuda, cin, cout):
    from o3dml_amd import layers
    pos = _voxels(4000, 24, cin)
    torch.manual_seed(0)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=True).to(cuda)
    torch.nn.init.normal_(conv.bias)
    feat = torch.randn(len(pos), cin, device=cuda)
    p = torch.from_numpy(pos).to(cuda)
    out = conv(feat, p, p, 1.0)
    # oracle rulebook
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    nb = conv.nns(p, p, 1.5)
    assert np.array_equal(nb.neighbors_index.cpu().numpy(), oi)
    from o3dml_amd import sparse_conv as sc
    kid = sc.kernel_index(p, p, nb.neighbors_index, nb.neighbors_row_splits, [3, 3, 3], 1.0)
    assert np.array_equal(kid.cpu().numpy(), ok)
    ref = O.sparse_conv(conv.kernel.detach().cpu().numpy(), feat.cpu().numpy(), oi, ok, ors)
    ref = ref + conv.bias.detach().cpu().numpy()
    _close(out.detach().cpu().numpy(), ref)
    t64, mag = _truth64(conv.kernel.detach().cpu().numpy(), feat.cpu().numpy(), oi, ok, ors,
                        conv.bias.detach().cpu().numpy())
    _close_elem(out.detach().cpu().numpy(), t64, mag)


@pytest.mark.parametrize("n,ext,cin,cout", [(300, 9, 128, 160), (120, 9, 192, 224), (2000, 14, 64, 64)])
def test_deep_level_conv_split_k(cuda, n, ext, cin, cout):
    """Few output rows and wide channels (SparseConvUnet's deep levels): the
    GEMM splits its (offset, Cin-chunk) stages over 13-40 grid slabs and
    split_reduce_kernel sums them — per element against the float64 truth,
    plain and with the fused eval prologue (BN + ReLU gathered) and residual
    epilogue."""
    from o3dml_amd import layers
    pos = _voxels(n, ext, n)
    torch.manual_seed(1)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=True).to(cuda)
    torch.nn.init.normal_(conv.bias)
    feat = torch.randn(len(pos), cin, device=cuda)
    p = torch.from_numpy(pos).to(cuda)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    W = conv.kernel.detach().cpu().numpy()
    with torch.no_grad():
        out = conv(feat, p, p, 1.0)
    _close_elem(out.cpu().numpy(), *_truth64(W, feat.cpu().numpy(), oi, ok, ors, conv.bias.detach().cpu().numpy()))
    scale = torch.rand(cin, device=cuda) + 0.5
    shift = torch.randn(cin, device=cuda) * 0.1
    res = torch.randn(len(pos), cout, device=cuda)
    with torch.no_grad():
        fused = conv.forward_fused(feat, p, p, 1.0, pre=(scale, shift), residual=res)
    x = torch.relu(feat * scale + shift).cpu().numpy()
    t64, mag = _truth64(W, x, oi, ok, ors, conv.bias.detach().cpu().numpy())
    _close_elem(fused.cpu().numpy(), t64 + res.cpu().numpy(), mag + np.abs(res.cpu().numpy()))


def test_strided_and_transposed_conv(cuda):
    """Convolution 2^3 stride 2 (calculate_grid) and its DeConvolution adjoint
    (sparseconvnet.py:388-482)."""
    from o3dml_amd import layers, sparse_conv as sc
    pos = _voxels(5000, 30, 3)
    p = torch.from_numpy(pos).to(cuda)
    # calculate_grid (sparseconvnet.py:388-401), reference torch code
    filt = torch.tensor([[-1, -1, -1], [-1, -1, 0], [-1, 0, -1], [-1, 0, 0], [0, -1, -1], [0, -1, 0], [0, 0, -1],
                         [0, 0, 0]], device=cuda)
    op = p.long().repeat(1, 8).reshape(-1, 3) + filt.repeat(p.shape[0], 1)
    op = op[op.min(1).values >= 0]
    op = op[(~((op.long() % 2).bool()).any(1))]
    out_pos = (torch.unique(op, dim=0) + 0.5).float()
    conv = layers.SparseConv(16, 32, [2, 2, 2], use_bias=False, offset=torch.full((3,), -0.5)).to(cuda)
    feat = torch.randn(len(pos), 16, device=cuda)
    out = conv(feat, p, out_pos, 1.0)
    q = (out_pos + 0.5).cpu().numpy()
    oi, ors, _ = O.fixed_radius_search(pos, q, 1.0, metric="Linf")
    ok = O.kernel_index(pos, q, oi, ors, [2, 2, 2], 1.0)
    assert (np.diff(ors) <= 8).all() and (np.diff(ors) >= 1).all()
    ref = O.sparse_conv(conv.kernel.detach().cpu().numpy(), feat.cpu().numpy(), oi, ok, ors)
    _close(out.detach().cpu().numpy(), ref)
    _close_elem(out.detach().cpu().numpy(), *_truth64(conv.kernel.detach().cpu().numpy(), feat.cpu().numpy(), oi,
                                                      ok, ors))
    # transposed: coarse (2*coarse_pos in fine coords) -> fine positions
    coarse = out_pos / 2
    deconv = layers.SparseConvTranspose(32, 16, [2, 2, 2], use_bias=False, offset=torch.full((3,), -0.5)).to(cuda)
    cf = torch.randn(len(coarse), 32, device=cuda)
    fo = deconv(cf, 2 * coarse, p, 1.0)
    qi = (p - 0.5).cpu().numpy()
    ti, trs, _ = O.fixed_radius_search((2 * coarse).cpu().numpy(), qi, 1.0, metric="Linf")
    tk = O.kernel_index((2 * coarse).cpu().numpy(), qi, ti, trs, [2, 2, 2], 1.0, mirror=True)
    assert (np.diff(trs) == 1).all()  # every fine voxel has exactly one parent
    ref = O.sparse_conv(deconv.kernel.detach().cpu().numpy(), cf.cpu().numpy(), ti, tk, trs)
    _close(fo.detach().cpu().numpy(), ref)
    _close_elem(fo.detach().cpu().numpy(), *_truth64(deconv.kernel.detach().cpu().numpy(), cf.cpu().numpy(), ti,
                                                     tk, trs))
    # adjointness: <conv(x), y> == <x, deconv_W(y)> with the same weights
    deconv.kernel.data.copy_(conv.kernel.data.transpose(3, 4))
    lhs = (conv(feat, p, out_pos, 1.0) * cf).sum()
    rhs = (feat * deconv(cf, 2 * coarse, p, 1.0)).sum()
    assert abs(float(lhs) - float(rhs)) <= 1e-4 * abs(float(lhs)) + 1e-3


@pytest.mark.parametrize("cin,cout", [(32, 32), (3, 48), (64, 64)])
def test_sparse_conv_backward(cuda, cin, cout):
    from o3dml_amd import ops
    pos = _voxels(3000, 20, 7 + cin)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    W = torch.randn(3, 3, 3, cin, cout, dtype=torch.float64) * 0.1
    x = torch.randn(len(pos), cin, dtype=torch.float64)
    g = torch.randn(len(pos), cout, dtype=torch.float64)
    Wd = W.float().to(cuda).requires_grad_()
    xd = x.float().to(cuda).requires_grad_()
    out = ops.sparse_conv(Wd, xd, torch.empty(0), torch.from_numpy(oi), torch.from_numpy(ok), torch.empty(0),
                          torch.from_numpy(ors))
    out.backward(g.float().to(cuda))
    W64, x64 = W.clone().requires_grad_(), x.clone().requires_grad_()
    ref = _csr_conv64(W64, x64, torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ors))
    ref.backward(g)
    _close(out.detach().cpu().numpy(), ref.detach().numpy())
    _close(xd.grad.cpu().numpy(), x64.grad.numpy())
    # per element vs float64: the forward, dIn (a conv of g with the
    # transposed filters over the same pairs) and dW (per filter entry a sum
    # over pairs of x * g) with their own term-magnitude sums
    mag = _csr_conv64(W.abs(), x.abs(), torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ors))
    _close_elem(out.detach().cpu().numpy(), ref.detach().numpy(), mag.numpy())
    Wa, xa = W.abs().clone().requires_grad_(), x.abs().clone().requires_grad_()
    _csr_conv64(Wa, xa, torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ors)).backward(g.abs())
    _close_elem(xd.grad.cpu().numpy(), x64.grad.numpy(), xa.grad.numpy())
    _close_elem(Wd.grad.cpu().numpy(), W64.grad.numpy(), Wa.grad.numpy())
    _close(Wd.grad.cpu().numpy(), W64.grad.numpy())


def test_sparse_conv_importance_normalize(cuda):
    from o3dml_amd import ops
    pos = _voxels(2000, 16, 21)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    rng = np.random.default_rng(5)
    W = rng.standard_normal((3, 3, 3, 8, 24)).astype(np.float32)
    x = rng.standard_normal((len(pos), 8)).astype(np.float32)
    ii = rng.random(len(pos)).astype(np.float32)
    ni = rng.random(len(oi)).astype(np.float32)
    out = ops.sparse_conv(torch.from_numpy(W).to(cuda), torch.from_numpy(x).to(cuda), torch.from_numpy(ii),
                          torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ni), torch.from_numpy(ors),
                          normalize=True)
    ref = O.sparse_conv(W, x, oi, ok, ors, inp_importance=ii, neighbors_importance=ni, normalize=True)
    _close(out.cpu().numpy(), ref)


@pytest.mark.parametrize("case", ["submanifold", "strided", "transposed"])
def test_lattice_rulebook_equals_search_rulebook(cuda, case):
    """The lattice rulebook (voxel hash) and the Linf fixed-radius-search
    rulebook give the same dense kernel map, so outputs and gradients agree
    bit for bit."""
    from o3dml_amd import layers
    from o3dml_amd.ops import calculate_grid
    pos = torch.from_numpy(_voxels(5000, 30, 11)).to(cuda)
    torch.manual_seed(1)
    if case == "submanifold":
        conv = layers.SparseConv(16, 24, [3, 3, 3]).to(cuda)
        inp, outp = pos, pos
    elif case == "strided":
        conv = layers.SparseConv(16, 24, [2, 2, 2], offset=torch.full((3,), -0.5)).to(cuda)
        inp, outp = pos, calculate_grid(pos)
    else:
        conv = layers.SparseConvTranspose(16, 24, [2, 2, 2], offset=torch.full((3,), -0.5)).to(cuda)
        inp, outp = calculate_grid(pos), pos
    feat = torch.randn(inp.shape[0], 16, device=cuda, requires_grad=True)
    outs, grads = [], []
    for lattice in (True, False):
        conv.lattice_rulebook = lattice
        conv.kernel.grad = None
        feat.grad = None
        out = conv(feat, inp, outp, 1.0)
        out.square().sum().backward()
        outs.append(out.detach())
        grads.append((feat.grad.clone(), conv.kernel.grad.clone()))
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


def test_lattice_rulebook_falls_back_off_lattice(cuda):
    from o3dml_amd import layers, sparse_conv as sc
    pos = _voxels(3000, 20, 5)
    jitter = pos + np.random.default_rng(0).uniform(-0.2, 0.2, pos.shape).astype(np.float32)
    p = torch.from_numpy(jitter).to(cuda)
    conv = layers.SparseConv(8, 8, [3, 3, 3]).to(cuda)
    feat = torch.randn(len(pos), 8, device=cuda)
    with torch.no_grad():
        assert sc.conv_lattice(conv.kernel, conv.bias, feat, p, p, 1.0) is None  # not a lattice
        out = conv(feat, p, p, 1.0)
    oi, ors, _ = O.fixed_radius_search(jitter, jitter, 1.5, metric="Linf")
    ok = O.kernel_index(jitter, jitter, oi, ors, [3, 3, 3], 1.0)
    ref = O.sparse_conv(conv.kernel.detach().cpu().numpy(), feat.cpu().numpy(), oi, ok, ors)
    _close(out.cpu().numpy(), ref + conv.bias.detach().cpu().numpy())


@pytest.mark.parametrize("cin,cout", [(32, 32), (64, 128), (3, 48)])
def test_bf16_split_products_match_exact_f32(cuda, cin, cout):
    """Product precisions of the gather-GEMMs against a float64 reference:
    bf16x6 (each f32 operand as hi + mid + lo bf16, six products; opt-in)
    must be as accurate as the exact f32-input MFMA kernel (the default) (within a few times
    its own f32 rounding error); bf16x3 (two terms, three products) within the
    north-star 1e-4.  Forward, input gradient and filter gradient; features
    span six decades of magnitude across channels."""
    from o3dml_amd import _lib, ops
    lib = _lib.load()
    pos = _voxels(3000, 20, 11 + cin)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    gen = torch.Generator().manual_seed(cin + cout)
    W = torch.randn(3, 3, 3, cin, cout, dtype=torch.float64, generator=gen) * 0.1
    x = torch.randn(len(pos), cin, dtype=torch.float64, generator=gen) * \
        10.0 ** torch.randint(-3, 4, (1, cin), generator=gen).double()
    g = torch.randn(len(pos), cout, dtype=torch.float64, generator=gen)
    W64, x64 = W.clone().requires_grad_(), x.clone().requires_grad_()
    ref = _csr_conv64(W64, x64, torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ors))
    ref.backward(g)
    refs = [ref.detach().numpy(), x64.grad.numpy(), W64.grad.numpy()]
    errs = {}
    prev = lib.o3dml_sparse_conv_set_exact(-1)
    assert prev in (0, 1, 2)
    assert lib.o3dml_sparse_conv_set_exact(3) == -1 and lib.o3dml_sparse_conv_set_exact(-1) == prev
    try:
        for mode in (0, 1, 2):
            lib.o3dml_sparse_conv_set_exact(mode)
            Wd = W.float().to(cuda).requires_grad_()
            xd = x.float().to(cuda).requires_grad_()
            out = ops.sparse_conv(Wd, xd, torch.empty(0), torch.from_numpy(oi), torch.from_numpy(ok),
                                  torch.empty(0), torch.from_numpy(ors))
            out.backward(g.float().to(cuda))
            got = [out.detach().cpu().numpy(), xd.grad.cpu().numpy(), Wd.grad.cpu().numpy()]
            errs[mode] = [np.abs(a - b).max() / (np.abs(b).max() + 1e-30) for a, b in zip(got, refs)]
            for a, b in zip(got, refs):
                _close(a, b)
    finally:
        lib.o3dml_sparse_conv_set_exact(prev)
    for e6, e1 in zip(errs[0], errs[1]):
        assert e6 <= 3 * e1 + 1e-7, (errs[0], errs[1])


def test_default_precision_is_exact_f32_and_keeps_infinities(cuda):
    """The default product precision is the exact f32-input MFMA (mode 1):
    a +-inf feature gives the IEEE result (+-inf, or NaN only where the
    exact arithmetic itself makes one: inf * 0, inf - inf), and finite
    outputs are unaffected."""
    from o3dml_amd import _lib, ops
    lib = _lib.load()
    assert lib.o3dml_sparse_conv_set_exact(-1) == 1
    pos = _voxels(2000, 16, 6)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    gen = torch.Generator().manual_seed(4)
    W = torch.rand(3, 3, 3, 32, 32, generator=gen) + 0.05  # positive weights: inf stays inf
    x = torch.rand(len(pos), 32, generator=gen)
    x[11, 5] = float("inf")
    out = ops.sparse_conv(W.to(cuda), x.to(cuda), torch.empty(0), torch.from_numpy(oi), torch.from_numpy(ok),
                          torch.empty(0), torch.from_numpy(ors)).cpu().numpy()
    hit = np.array([np.isin(oi[ors[q]:ors[q + 1]], [11]).any() for q in range(len(pos))])
    assert hit.any() and np.isposinf(out[hit]).all()
    assert np.isfinite(out[~hit]).all()


def test_bf16_split_large_and_nonfinite_inputs(cuda):
    """The bf16x6 split's range (DESIGN §5 "Product precision"): features up to
    1e30 stay within the f32 tolerance of float64 (hi carries the exponent,
    so magnitude costs no bits); a non-finite feature makes exactly the
    outputs that gather its row non-finite (inf - inf in the split turns the
    exact path's +-inf into NaN there — the documented deviation; exact mode,
    o3dml_sparse_conv_set_exact(1), keeps IEEE infinities), every other output
    stays equal to the exact kernel's within its rounding."""
    from o3dml_amd import _lib, ops
    lib = _lib.load()
    pos = _voxels(2000, 16, 5)
    oi, ors, _ = O.fixed_radius_search(pos, pos, 1.5, metric="Linf")
    ok = O.kernel_index(pos, pos, oi, ors, [3, 3, 3], 1.0)
    gen = torch.Generator().manual_seed(3)
    W = torch.randn(3, 3, 3, 32, 32, dtype=torch.float64, generator=gen) * 0.1
    x = torch.randn(len(pos), 32, dtype=torch.float64, generator=gen) * 1e30
    ref = _csr_conv64(W, x, torch.from_numpy(oi), torch.from_numpy(ok), torch.from_numpy(ors)).numpy()
    args = (torch.empty(0), torch.from_numpy(oi), torch.from_numpy(ok), torch.empty(0), torch.from_numpy(ors))
    prev = lib.o3dml_sparse_conv_set_exact(-1)
    try:
        lib.o3dml_sparse_conv_set_exact(0)
        got = ops.sparse_conv(W.float().to(cuda), x.float().to(cuda), *args).cpu().numpy()
        _close(got, ref)
        xi = x.float().clone()
        xi[7, 3], xi[100, 0] = float("inf"), float("-inf")
        res = {}
        for mode in (0, 1):
            lib.o3dml_sparse_conv_set_exact(mode)
            res[mode] = ops.sparse_conv(W.float().to(cuda), xi.to(cuda), *args).cpu().numpy()
    finally:
        lib.o3dml_sparse_conv_set_exact(prev)
    hit = np.zeros(len(pos), bool)
    for q in range(len(pos)):
        hit[q] = np.isin(oi[ors[q]:ors[q + 1]], [7, 100]).any()
    assert hit.any()
    assert not np.isfinite(res[0][hit]).all(axis=1).any() and not np.isfinite(res[1][hit]).all(axis=1).any()
    assert np.isfinite(res[0][~hit]).all() and np.isfinite(res[1][~hit]).all()
    scale = np.abs(res[1][~hit]).max()
    assert np.abs(res[0][~hit] - res[1][~hit]).max() <= 1e-6 * scale


@pytest.mark.parametrize("cin", [8, 3])
@pytest.mark.parametrize("normalize,importance", [(False, False), (True, False), (True, True)])
def test_duplicate_kernel_indices(cuda, normalize, importance, cin):
    """Off-lattice positions: several neighbours of one output share a kernel
    index (Open3D sums every pair).  The pairs are split into dense-map layers
    (sparse_conv._conv_layers); forward vs the oracle (which sums the CSR pairs
    directly), filter and feature gradients vs float64 autograd of the CSR
    convolution, through layers.SparseConv's search rulebook.  cin 3: the
    narrow-input VALU kernel (small_cin_gemm_kernel) with row / pair scales."""
    from o3dml_amd import layers, ops
    rng = np.random.default_rng(31)
    pos = (rng.random((1500, 3)) * 12).astype(np.float32)  # continuous positions: ~1.7 points per voxel
    inp = torch.from_numpy(pos).to(cuda)
    conv = layers.SparseConv(cin, 16, [3, 3, 3], use_bias=True, normalize=normalize).to(cuda)
    torch.nn.init.normal_(conv.bias)
    conv.lattice_rulebook = False
    nb, kidx = conv._rulebook(inp, inp, 1.0, None, False, 1.0)
    idx, rs, kid = (nb.neighbors_index.cpu().numpy(), nb.neighbors_row_splits.cpu().numpy(), kidx.cpu().numpy())
    o = np.repeat(np.arange(len(rs) - 1), np.diff(rs))
    assert len(np.unique(o * 27 + kid)) < len(kid)  # duplicates present
    x = torch.randn((1500, cin), device=cuda, requires_grad=True)
    # per-input-point importance, gathered per pair (the layer's inp_importance)
    pimp = torch.rand(1500, device=cuda) if importance else None
    nimp = pimp[nb.neighbors_index.long()] if importance else None
    W = conv.kernel
    out = ops.sparse_conv(W, x, None, nb.neighbors_index, kidx, nimp, nb.neighbors_row_splits,
                          normalize=normalize) + conv.bias
    ref = O.sparse_conv(W.detach().cpu().numpy(), x.detach().cpu().numpy(), idx, kid, rs,
                        neighbors_importance=None if nimp is None else nimp.cpu().numpy(),
                        normalize=normalize) + conv.bias.detach().cpu().numpy()
    _close(out.detach().cpu().numpy(), ref)
    # the layer path (bias in the epilogue, normalisation after the layer sum)
    ref_l = ref if not importance else O.sparse_conv(
        W.detach().cpu().numpy(), x.detach().cpu().numpy(), idx, kid, rs, inp_importance=pimp.cpu().numpy(),
        normalize=normalize) + conv.bias.detach().cpu().numpy()
    _close(conv(x, inp, inp, 1.0, inp_importance=pimp).detach().cpu().numpy(), ref_l)
    go = torch.randn_like(out)
    gW, gx = torch.autograd.grad(out, (W, x), go)
    W64 = W.detach().cpu().double().requires_grad_(True)
    x64 = x.detach().cpu().double().requires_grad_(True)
    Wf = W64.reshape(27, cin, 16)
    contrib = torch.einsum("pc,pcd->pd", x64[torch.from_numpy(idx).long()], Wf[torch.from_numpy(kid).long()])
    if importance:
        contrib = contrib * nimp.cpu().double()[:, None]
    r64 = torch.zeros((len(rs) - 1, 16), dtype=torch.float64).index_add_(0, torch.from_numpy(o), contrib)
    if normalize:
        w = nimp.cpu().double() if importance else torch.ones(len(idx), dtype=torch.float64)
        den = torch.zeros(len(rs) - 1, dtype=torch.float64).index_add_(0, torch.from_numpy(o), w)
        r64 = r64 / torch.where(den != 0, den, torch.ones_like(den))[:, None]
    gW64, gx64 = torch.autograd.grad(r64, (W64, x64), go.cpu().double())
    _close(gW.cpu().numpy(), gW64.numpy())
    _close(gx.cpu().numpy(), gx64.numpy())


@pytest.mark.parametrize("cin,cout", [(32, 32), (16, 48), (64, 64), (128, 128), (96, 224)])
def test_presplit_operands_bitwise_equal(cuda, cin, cout):
    """The presplit GEMM (operand hi/mid/lo planes made once per call,
    implicit_gemm_split_kernel) against the in-kernel split
    (implicit_gemm_lds/shared_kernel): the same split values and MFMA order,
    so forward, dIn and dW are bitwise identical, in bf16x6 and bf16x3."""
    from o3dml_amd import _lib, layers
    lib = _lib.load()
    vox = torch.from_numpy(_voxels(30000, 40, 3)).to(cuda)
    torch.manual_seed(0)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=True).to(cuda)
    x = torch.randn((vox.shape[0], cin), device=cuda, requires_grad=True)
    go = torch.randn((vox.shape[0], cout), device=cuda)
    prev_mode = lib.o3dml_sparse_conv_set_exact(-1)
    prev = lib.o3dml_sparse_conv_set_presplit(-1)
    try:
        for mode in (0, 2):
            lib.o3dml_sparse_conv_set_exact(mode)
            res = []
            for on in (1, 0):
                lib.o3dml_sparse_conv_set_presplit(on)
                out = conv(x, vox, vox, 1.0)
                res.append((out,) + torch.autograd.grad(out, (x, conv.kernel), go))
            for a, b in zip(*res):
                assert torch.equal(a, b), (mode, cin, cout)
    finally:
        lib.o3dml_sparse_conv_set_presplit(prev)
        lib.o3dml_sparse_conv_set_exact(prev_mode)


@pytest.mark.parametrize("cin,cout", [(32, 32), (64, 32), (32, 16), (96, 48), (16, 32)])
def test_split_filters_bitwise_equal(cuda, cin, cout):
    """Filters split into bf16 hi / mid / lo once per call (split_filters_kernel,
    the BS form of implicit_gemm_lds_kernel) against the per-stage split: the
    same bf16 terms in the same MFMA order, so the forward is bitwise
    identical; the SparseConvUnet eval (prologue + residual) too."""
    from o3dml_amd import _lib, layers
    from o3dml_amd.sparseconvnet import SparseConvUnet
    import types
    lib = _lib.load()
    vox = torch.from_numpy(_voxels(30000, 40, 3)).to(cuda)
    torch.manual_seed(0)
    conv = layers.SparseConv(cin, cout, [3, 3, 3], use_bias=True).to(cuda)
    x = torch.randn((vox.shape[0], cin), device=cuda)
    m = SparseConvUnet(multiplier=16, residual_blocks=True, conv_block_reps=1, num_classes=5).to(cuda).eval()
    g = torch.Generator().manual_seed(1)
    pos = (torch.rand((20000, 3), generator=g) * 30).to(cuda)
    inp = types.SimpleNamespace(point=[pos], feat=[torch.rand((20000, 3), generator=g).to(cuda)],
                                batch_lengths=[20000])
    prev = lib.o3dml_sparse_conv_set_bsplit(-1)
    try:
        res = []
        for on in (1, 0):
            lib.o3dml_sparse_conv_set_bsplit(on)
            with torch.no_grad():
                res.append((conv(x, vox, vox, 1.0), m(inp)))
        for a, b in zip(*res):
            assert torch.equal(a, b), (cin, cout)
    finally:
        lib.o3dml_sparse_conv_set_bsplit(prev)


def test_presplit_fused_eval_bitwise_equal(cuda):
    """SparseConvUnet eval (BN + ReLU prologue folded into the presplit
    planes, residual epilogue): presplit on / off give identical logits."""
    from o3dml_amd import _lib
    from o3dml_amd.sparseconvnet import SparseConvUnet
    import types
    lib = _lib.load()
    torch.manual_seed(0)
    m = SparseConvUnet(multiplier=16, residual_blocks=True, conv_block_reps=1, num_classes=5).to(cuda).eval()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
    g = torch.Generator().manual_seed(1)
    pos = (torch.rand((20000, 3), generator=g) * 30).to(cuda)
    inp = types.SimpleNamespace(point=[pos], feat=[torch.rand((20000, 3), generator=g).to(cuda)],
                                batch_lengths=[20000])
    prev = lib.o3dml_sparse_conv_set_presplit(-1)
    try:
        outs = []
        for on in (1, 0):
            lib.o3dml_sparse_conv_set_presplit(on)
            with torch.no_grad():
                outs.append(m(inp))
        assert torch.equal(outs[0], outs[1])
    finally:
        lib.o3dml_sparse_conv_set_presplit(prev)


def test_split_k_last_wave_finish_bitwise(cuda, tmp_path):
    """Split-K GEMMs (deep SparseConvUnet levels) optionally finish in the
    last-arriving wave of each tile (O3DML_GEMM_FUSED_REDUCE=1) instead of a
    split_reduce_kernel launch: same slab order and epilogue, so
    bit-identical (child processes: the switch is read once).  Eval (BN/ReLU prologue +
    residual epilogue) and a training forward + backward (dIn split too)."""
    import os
    import subprocess
    import sys
    code = ("import sys, types, torch; sys.path.insert(0, 'open3d-ml_amd')\n"
            "from o3dml_amd.sparseconvnet import SparseConvUnet\n"
            "torch.manual_seed(0)\n"
            "m = SparseConvUnet(multiplier=16, residual_blocks=True, conv_block_reps=1, num_classes=5).cuda()\n"
            "g = torch.Generator().manual_seed(1)\n"
            "pos = (torch.rand((30000, 3), generator=g) * torch.tensor([200., 200., 30.])).cuda()\n"
            "inp = types.SimpleNamespace(point=[pos], feat=[torch.rand((30000, 3), generator=g).cuda()],"
            " batch_lengths=[30000])\n"
            "m.eval()\n"
            "with torch.no_grad():\n"
            "    a = m(inp)\n"
            "m.train()\n"
            "out = m(inp)\n"
            "out.square().sum().backward()\n"
            "torch.save([a.cpu(), out.detach().cpu()] + [p.grad.cpu() for p in m.parameters() if p.grad is not None],"
            " sys.argv[1])\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for flag in ("1", "0"):
        path = str(tmp_path / f"sc_reduce_{flag}.pt")
        env = dict(os.environ, O3DML_GEMM_FUSED_REDUCE=flag)
        subprocess.run([sys.executable, "-c", code, path], check=True, env=env, cwd=root, timeout=180)
        outs.append(torch.load(path, weights_only=True))
    assert len(outs[0]) == len(outs[1]) > 2
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_gemm_schedules_bitwise(cuda, tmp_path):
    """The GEMM's work schedules change no bits: the persistent grid with the
    next tile prefetched (O3DML_GEMM_PERSIST, default 1) against one wave per
    item, and the tile-order map copy (O3DML_GEMM_TILE_MAP, default 1) against
    reading the map through the order — every row's (offset, Cin) stages and
    split partition are the same (child processes: the switches are read once).
    A C4-sized room (88k voxels, cached tile-ordered map, so the persistent grid
    engages), 32 -> 32 and 32 -> 64 forward, dIn and dW."""
    import os
    import subprocess
    import sys
    code = ("import sys, torch; sys.path[:0] = ['.', 'open3d-ml_amd']\n"
            "import bench\n"
            "from o3dml_amd import layers, sparse_conv as sc\n"
            "pos = torch.from_numpy(bench.make_room(0)[0]).cuda()\n"
            "res = []\n"
            "for cout in (32, 64):\n"
            "    torch.manual_seed(0)\n"
            "    conv = layers.SparseConv(32, cout, [3, 3, 3], use_bias=False).cuda()\n"
            "    x = torch.rand((pos.shape[0], 32), device='cuda', requires_grad=True)\n"
            "    with sc.rulebook_cache():\n"
            "        out = conv(x, pos, pos, 1.0)\n"
            "        out.square().sum().backward()\n"
            "    res += [out.detach().cpu(), x.grad.cpu(), conv.kernel.grad.cpu()]\n"
            "torch.save(res, sys.argv[1])\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for i, extra in enumerate(({}, {"O3DML_GEMM_PERSIST": "0"}, {"O3DML_GEMM_TILE_MAP": "0"})):
        path = str(tmp_path / f"sched_{i}.pt")
        env = dict(os.environ, **extra)
        subprocess.run([sys.executable, "-c", code, path], check=True, env=env, cwd=root, timeout=180)
        outs.append(torch.load(path, weights_only=True))
    for other in outs[1:]:
        assert len(other) == len(outs[0]) == 6
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)


def test_transposed_conv_normalize(cuda):
    """layers.SparseConvTranspose(normalize=True): every input's contribution
    divided by its number of output neighbours (ops.sparse_conv_transpose's
    inp_neighbors_* relation), against a float64 restatement over the same
    rulebook; the gradients through the registered backward."""
    from o3dml_amd import layers
    vox = torch.from_numpy(_voxels(4000, 24, 8)).to(cuda)
    coarse = torch.unique(torch.floor(vox / 2), dim=0) * 2 + 1.0  # stride-2 lattice
    torch.manual_seed(0)
    conv = layers.SparseConvTranspose(16, 24, [3, 3, 3], use_bias=True, normalize=True).to(cuda)
    torch.nn.init.normal_(conv.bias)
    x = torch.randn((coarse.shape[0], 16), device=cuda, requires_grad=True)
    out = conv(x, coarse, vox, 2.0)
    nb, kidx = conv._rulebook(coarse, vox, 2.0, None, True, -1.0)
    idx = nb.neighbors_index.long().cpu()
    rs = nb.neighbors_row_splits.cpu()
    o = torch.repeat_interleave(torch.arange(vox.shape[0]), rs[1:] - rs[:-1])
    cnt = torch.bincount(idx, minlength=coarse.shape[0]).double()
    W = conv.kernel.detach().double().cpu().reshape(27, 16, 24)
    x64 = x.detach().double().cpu()
    contrib = torch.einsum("pc,pcd->pd", x64[idx] / cnt[idx][:, None], W[kidx.long().cpu()])
    ref = torch.zeros((vox.shape[0], 24), dtype=torch.float64).index_add_(0, o, contrib) + conv.bias.detach().double().cpu()
    _close(out.detach().cpu().numpy(), ref.numpy())
    go = torch.randn_like(out)
    gx, = torch.autograd.grad(out, x, go)
    x64r = x64.clone().requires_grad_(True)
    contrib = torch.einsum("pc,pcd->pd", x64r[idx] / cnt[idx][:, None], W[kidx.long().cpu()])
    r = torch.zeros((vox.shape[0], 24), dtype=torch.float64).index_add_(0, o, contrib)
    gx64, = torch.autograd.grad(r, x64r, go.double().cpu())
    _close(gx.cpu().numpy(), gx64.numpy())


def test_out_of_range_neighbour_index_and_map_entry(cuda):
    """A neighbour index past the input features raises RuntimeError (the
    map build drops the pair and flags it, status bit 3) instead of reading
    past the features; and a map entry corrupted past the operand (the
    buffer-resource GEMM, cin % 32 == 0) reads zeros: its output row equals
    the row with that pair removed (num_records = the operand's true size)."""
    from o3dml_amd import _lib, layers, sparse_conv as sc
    from o3dml_amd._util import ptr, stream_handle, workspace
    vox = torch.from_numpy(_voxels(3000, 16, 4)).to(cuda)
    conv = layers.SparseConv(32, 32, [3, 3, 3], use_bias=False).to(cuda)
    conv.lattice_rulebook = False
    nb, kidx = conv._rulebook(vox, vox, 1.0, None, False, 1.0)
    n = vox.shape[0]
    x = torch.randn((n, 32), device=cuda)
    bad = nb.neighbors_index.clone()
    bad[5] = n + 7
    with pytest.raises(RuntimeError, match="neighbors_index out of range"):
        sc.sparse_conv(conv.kernel, x, None, bad, kidx, None, nb.neighbors_row_splits)
    lib = _lib.load()
    dev = x.device
    st = stream_handle(dev)
    W = conv.kernel.detach().contiguous()
    K = 27
    outs = []
    for corrupt in (None, n + 100000, -1):
        mws, n_out = sc._build_map(nb.neighbors_index, kidx, None, nb.neighbors_row_splits, n, K, False, None,
                                   False, False, dev, st)
        m = mws[:n_out * K * 4].view(torch.int32)
        o = 11
        k = int(torch.nonzero(m[o * K:(o + 1) * K] >= 0)[0])
        if corrupt is not None:
            m[o * K + k] = corrupt
        out = torch.empty((n_out, 32), device=dev)
        fws = workspace(lib.o3dml_sparse_conv_forward_workspace_size(n_out, n, K, 32, 32), dev)
        _lib.call("o3dml_sparse_conv_forward", ptr(W), K, 32, 32, ptr(x), n, None, 0, 0, None, n_out, ptr(out),
                  ptr(mws), mws.numel(), ptr(fws), fws.numel(), st)
        outs.append(out)
    assert torch.equal(outs[1], outs[2])  # past the operand == absent
    assert not torch.equal(outs[0][11], outs[2][11]) and torch.equal(outs[0][12:], outs[2][12:])


@pytest.mark.parametrize("ks", [2, 3])
@pytest.mark.parametrize("want_grad", [False, True])
def test_transpose_map_derived_from_conv_map(cuda, want_grad, ks):
    """In a rulebook_cache scope a SparseConvTranspose whose SparseConv
    partner (positions swapped, same kernel / offset) is cached takes the
    partner's map inverted (o3dml_sparse_conv_transpose_map) instead of
    building its own: forward (and, with gradients, dIn / dW) bit-identical
    to the transpose built on its own.  The derivation is counted by the
    scope (scope.derived), so a silent fallback to an own-built map fails;
    3^3 also runs the tile order on the derived map."""
    from o3dml_amd import layers, ops, sparse_conv as sc
    pos = _voxels(6000, 30, 41)
    p = torch.from_numpy(pos).to(cuda)
    outs = ops.calculate_grid(p)
    torch.manual_seed(0)
    off = torch.full((3,), -0.5) if ks == 2 else torch.zeros(3)
    conv = layers.SparseConv(16, 32, [ks] * 3, use_bias=False, offset=off).to(cuda)
    deconv = layers.SparseConvTranspose(32, 16, [ks] * 3, use_bias=False, offset=off).to(cuda)
    x = torch.randn(len(pos), 16, device=cuda)
    y = torch.randn(len(outs), 32, device=cuda)
    g = torch.randn(len(pos), 16, device=cuda)

    def run(derive):
        yy = y.clone().requires_grad_(want_grad)
        with torch.set_grad_enabled(want_grad), sc.rulebook_cache() as scope:
            if derive:
                conv(x, p, outs, 1.0)
            n_maps, n_derived = len(scope.maps), scope.derived
            out = deconv(yy, outs, p, 1.0)
            derived = len(scope.maps) - n_maps == 1 and scope.derived - n_derived == 1
            if want_grad:
                out.backward(g)
        return out.detach(), (yy.grad if want_grad else None), derived

    own, gown, own_derived = run(False)
    der, gder, derived = run(True)
    assert derived and not own_derived
    assert torch.equal(own, der)
    if want_grad:
        assert torch.equal(gown, gder)
