"""Run-to-run determinism: every hot-path
kernel the DESIGN calls deterministic gives BITWISE identical outputs when the
same inputs are run twice (fresh output buffers, same stream).  Float outputs
are compared as raw bit patterns (torch.equal on an int32 view), so -0/+0 and
NaN payload differences count as mismatches.

The three scatter-add backward kernels that use fp32 atomics like the
reference (KPConv feature gradient, KPFCNN max-pool gradient,
three_interpolate_grad) are checked in their deterministic mode
(torch.use_deterministic_algorithms(True): fixed-order gathers over a stable
radix-sorted inverse), which must also agree with the atomic path within fp32
rounding."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    t = t.detach()
    if t.dtype == torch.float32:
        return t.contiguous().view(torch.int32)
    if t.dtype == torch.float16:
        return t.contiguous().view(torch.int16)
    if t.dtype == torch.float64:
        return t.contiguous().view(torch.int64)
    return t


def _flatten(out):
    if isinstance(out, torch.Tensor):
        return [out]
    if isinstance(out, (tuple, list)):
        return [t for o in out for t in _flatten(o)]
    if hasattr(out, "_fields"):
        return [t for o in out for t in _flatten(o)]
    return []


def _twice(fn):
    a = _flatten(fn())
    b = _flatten(fn())
    assert len(a) == len(b) and len(a) > 0
    for i, (x, y) in enumerate(zip(a, b)):
        assert x.shape == y.shape and x.dtype == y.dtype, i
        assert torch.equal(_bits(x), _bits(y)), f"output {i} differs between identical runs"
    return a


@pytest.fixture
def deterministic():
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    yield
    torch.use_deterministic_algorithms(prev)


def _cloud(n, seed, extent=10.0):
    rng = np.random.default_rng(seed)
    return torch.from_numpy((rng.random((n, 3)) * extent).astype(np.float32))


def test_neighbor_searches_bitwise(cuda):
    from o3dml_amd import ops
    pts = _cloud(60000, 0).to(cuda)
    qs = _cloud(20000, 1).to(cuda)
    rs = torch.tensor([0, 30000, 60000])
    qrs = torch.tensor([0, 8000, 20000])
    _twice(lambda: ops.build_spatial_hash_table(pts, 0.4, rs))
    _twice(lambda: ops.fixed_radius_search(pts, qs, 0.4, rs, qrs, return_distances=True))
    _twice(lambda: ops.fixed_radius_search(pts, qs, 0.4, rs, qrs, metric="L1", ignore_query_point=True,
                                           return_distances=True))
    _twice(lambda: ops.knn_search(pts, qs, 16, rs, qrs, return_distances=True))
    _twice(lambda: ops.knn_search(pts, qs[:500], 300, rs, torch.tensor([0, 200, 500]), return_distances=True))
    radii = torch.rand(20000, device=cuda) * 0.5
    _twice(lambda: ops.radius_search(pts, qs, radii, rs, qrs, return_distances=True))


def test_pointnet2_and_voxel_ops_bitwise(cuda):
    from o3dml_amd import ops
    xyz = torch.rand((4, 4096, 3), device=cuda)
    _twice(lambda: ops.furthest_point_sampling(xyz, 1024))
    centers = xyz[:, :1024].contiguous()
    _twice(lambda: ops.ball_query(xyz, centers, 0.1, 32))
    d, idx = _twice(lambda: ops.three_nn(xyz, centers))
    w = 1.0 / (d + 1e-8)
    w = w / w.sum(2, keepdim=True)
    feats = torch.randn((4, 64, 1024), device=cuda)
    _twice(lambda: ops.three_interpolate(feats, idx, w))
    pts = _cloud(100000, 3, extent=40.0).to(cuda)
    _twice(lambda: ops.voxelize(pts, torch.tensor([0, 50000, 100000]), torch.tensor([0.2, 0.2, 0.2]),
                                torch.tensor([0.0, 0.0, 0.0]), torch.tensor([40.0, 40.0, 40.0]), 32, 40000))


def test_nms_bitwise(cuda):
    from o3dml_amd import ops
    rng = np.random.default_rng(5)
    ctr = rng.random((3000, 2)) * 60
    sz = rng.random((3000, 2)) * 3 + 1
    boxes = np.concatenate([ctr - sz / 2, ctr + sz / 2, rng.random((3000, 1)) * 3], 1).astype(np.float32)
    scores = rng.random(3000).astype(np.float32)
    scores[::7] = scores[0]  # ties
    b, s = torch.from_numpy(boxes).to(cuda), torch.from_numpy(scores).to(cuda)
    _twice(lambda: ops.nms(b, s, 0.3))


def test_sparse_conv_forward_backward_bitwise(cuda):
    """The gather-GEMM-scatter forward, dIn and dW (split-K slabs reduced in
    a fixed order, no atomics)."""
    from o3dml_amd import layers
    rng = np.random.default_rng(2)
    vox = np.unique(rng.integers(0, 48, (30000, 3)), axis=0).astype(np.float32) + 0.5
    pos = torch.from_numpy(vox).to(cuda)
    torch.manual_seed(0)
    conv = layers.SparseConv(32, 32, [3, 3, 3], use_bias=True).to(cuda)
    x = torch.randn((len(vox), 32), device=cuda, requires_grad=True)
    go = torch.randn((len(vox), 32), device=cuda)

    def run():
        out = conv(x, pos, pos, 1.0)
        gw, gx = torch.autograd.grad(out, (conv.kernel, x), go)
        return out, gw, gx
    _twice(run)


def test_kpconv_bitwise_and_deterministic_backward(cuda, deterministic):
    from o3dml_amd.kpconv import KPConv
    from o3dml_amd.kpfcnn import max_pool
    g = torch.Generator().manual_seed(0)
    s = torch.rand((6000, 3), generator=g)
    q = s[:5000] + 0.01 * torch.randn((5000, 3), generator=g)
    d = torch.cdist(q, s)
    nbr = torch.argsort(d, 1)[:, :40]
    nbr[d.gather(1, nbr) > 0.06] = 6000
    q, s, nbr = q.to(cuda), s.to(cuda), nbr.to(cuda)
    x = torch.randn((6000, 48), device=cuda, requires_grad=True)
    for infl, mode, deform in (("linear", "sum", False), ("gaussian", "sum", False), ("linear", "closest", False),
                               ("linear", "sum", True)):
        torch.manual_seed(1)
        conv = KPConv(15, 3, 48, 64, KP_extent=0.03, radius=0.05, KP_influence=infl, aggregation_mode=mode,
                      deformable=deform, modulated=deform).to(cuda)
        if deform:
            with torch.no_grad():
                conv.offset_conv.weights.normal_(0, 0.05)
                conv.offset_bias.normal_(0, 0.1)
        go = torch.randn((5000, 64), device=cuda)

        def run():
            out = conv(q, s, nbr, x)
            return (out,) + torch.autograd.grad(out, (x, conv.weights), go)
        det = _twice(run)
        torch.use_deterministic_algorithms(False)
        atom = run()
        torch.use_deterministic_algorithms(True, warn_only=True)
        for a, b in zip(det, atom):
            assert (a - b).abs().max() <= 1e-4 * (b.abs().max() + 1e-12), (infl, mode, deform)

    # KPFCNN max pooling gradient (duplicates in a row, shadow entries)
    xp = torch.randn((6000, 32), device=cuda, requires_grad=True)
    inds = torch.cat([nbr[:, :20], nbr[:, :3]], 1)
    gp = torch.randn((5000, 32), device=cuda)
    det = _twice(lambda: torch.autograd.grad(max_pool(xp, inds), xp, gp))
    torch.use_deterministic_algorithms(False)
    atom = torch.autograd.grad(max_pool(xp, inds), xp, gp)[0]
    torch.use_deterministic_algorithms(True, warn_only=True)
    assert (det[0] - atom).abs().max() <= 1e-5 * atom.abs().max()


def test_three_interpolate_grad_deterministic(cuda, deterministic):
    from o3dml_amd import ops
    xyz = torch.rand((2, 8192, 3), device=cuda)
    known = xyz[:, :1024].contiguous()
    d, idx = ops.three_nn(xyz, known)
    w = 1.0 / (d + 1e-8)
    w = w / w.sum(2, keepdim=True)
    go = torch.randn((2, 128, 8192), device=cuda)
    det = _twice(lambda: ops.three_interpolate_grad(go, idx, w, 1024))[0]
    torch.use_deterministic_algorithms(False)
    atom = ops.three_interpolate_grad(go, idx, w, 1024)
    torch.use_deterministic_algorithms(True, warn_only=True)
    # float64 reference
    ref = torch.zeros((2, 128, 1024), dtype=torch.float64, device=cuda)
    ref.scatter_add_(2, idx.long().reshape(2, 1, -1).expand(2, 128, -1),
                     (go.double()[:, :, :, None] * w.double()[:, None]).reshape(2, 128, -1))
    scale = ref.abs().max()
    assert (det.double() - ref).abs().max() <= 1e-5 * scale
    assert (atom.double() - ref).abs().max() <= 1e-5 * scale


def test_randla_dense_and_pipeline_bitwise(cuda):
    from o3dml_amd.randlanet import RandLANet, SemSegInference, dense_act
    for n, k, m in ((45056, 8, 16), (704, 768, 512), (2816, 256, 128)):
        a = torch.randn((n, k), device=cuda)
        w = torch.randn((m, k), device=cuda) / k ** 0.5
        b = torch.randn(m, device=cuda)
        _twice(lambda: dense_act(a, w, b, 0.2))
    torch.manual_seed(0)
    model = RandLANet(num_points=4096).to(cuda)
    rng = np.random.default_rng(1)
    pts = np.stack([rng.uniform(-20, 20, 20000), rng.uniform(-20, 20, 20000), rng.uniform(-2, 2, 20000)], 1)
    pts = torch.from_numpy(pts.astype(np.float32)).to(cuda)
    _twice(lambda: SemSegInference(model, seed=0).run(pts))
