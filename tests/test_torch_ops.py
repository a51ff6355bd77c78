"""torch.ops.open3d.* (o3dml_amd/torch_ops.py): the dispatcher registration
Open3D's op library provides (SURVEY.md §8b "Mechanism upstream").

CPU: every op is registered with Open3D's argument names, TorchScript
compiles callers, and the fake (meta) kernels give the output shapes/dtypes
(data-dependent sizes as symbolic sizes) without running anything.  GPU: the
registered ops return exactly what o3dml_amd.ops returns, and autograd through
torch.ops.open3d.sparse_conv / sparse_conv_transpose / three_interpolate
matches the gradients of the o3dml_amd autograd path."""
import numpy as np
import pytest
import torch

import o3dml_amd
from o3dml_amd import torch_ops

o3dml_amd.register_torch_ops()


def test_all_ops_registered_with_open3d_names():
    for name in torch_ops.OPS:
        op = getattr(torch.ops.open3d, name)
        assert op.default._schema.name == f"open3d::{name}"
    s = str(torch.ops.open3d.fixed_radius_search.default._schema)
    for arg in ("points_row_splits", "hash_table_cell_splits", "ScalarType index_dtype=3", 'str metric="L2"',
                "bool ignore_query_point=False", "bool return_distances=False"):
        assert arg in s
    s = str(torch.ops.open3d.sparse_conv.default._schema)
    assert "Tensor? inp_importance" in s and "Tensor neighbors_row_splits" in s


def test_shim_import_registers():
    import open3d.ml.torch  # noqa: F401
    assert hasattr(torch.ops.open3d, "knn_search")


@torch.jit.script
def _scripted_knn(p: torch.Tensor, q: torch.Tensor, rs: torch.Tensor, qrs: torch.Tensor):
    return torch.ops.open3d.knn_search(p, q, 8, rs, qrs)


@torch.jit.script
def _scripted_frs(p: torch.Tensor, rs: torch.Tensor):
    ht = torch.ops.open3d.build_spatial_hash_table(p, 0.1, rs, 1.0 / 64)
    return torch.ops.open3d.fixed_radius_search(p, p, 0.1, rs, rs, ht[2], ht[0], ht[1])


def test_torchscript_compiles_callers():
    g = str(_scripted_knn.graph)
    assert "open3d::knn_search" in g
    assert "open3d::fixed_radius_search" in str(_scripted_frs.graph)


def test_fake_kernels_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    from torch.fx.experimental.symbolic_shapes import ShapeEnv
    with FakeTensorMode(shape_env=ShapeEnv()):
        p = torch.empty((100, 3))
        rs = torch.tensor([0, 100])
        idx, nrs, dist = torch.ops.open3d.knn_search(p, p, 4, rs, rs, return_distances=True)
        assert nrs.shape == (101,) and idx.dtype == torch.int32 and dist.dtype == torch.float32
        f = torch.empty((3, 3, 3, 8, 16))
        x = torch.empty((100, 8))
        out = torch.ops.open3d.sparse_conv(f, x, None, torch.empty(50, dtype=torch.int32),
                                           torch.empty(50, dtype=torch.int32), None, torch.empty(41, dtype=torch.int64))
        assert out.shape == (40, 16)
        v = torch.ops.open3d.voxelize(p, rs, torch.ones(3), torch.zeros(3), torch.ones(3))
        assert v[0].dtype == torch.int32 and v[3].shape == (2,)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_registered_ops_equal_python_ops(cuda):
    from o3dml_amd import ops
    pts = torch.from_numpy(np.random.default_rng(0).random((3000, 3), dtype=np.float32)).to(cuda)
    rs = torch.tensor([0, 1000, 3000])
    a = torch.ops.open3d.knn_search(pts, pts, 16, rs, rs, torch.int64, "L2", False, True)
    b = ops.knn_search(pts, pts, 16, rs, rs, torch.int64, return_distances=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    ht = torch.ops.open3d.build_spatial_hash_table(pts, 0.05, rs, 1.0 / 64)
    a = torch.ops.open3d.fixed_radius_search(pts, pts, 0.05, rs, rs, ht[2], ht[0], ht[1])
    b = ops.fixed_radius_search(pts, pts, 0.05, rs, rs)
    assert torch.equal(a[0], b.neighbors_index) and torch.equal(a[1], b.neighbors_row_splits)
    radii = torch.full((3000,), 0.04, device=cuda)
    a = torch.ops.open3d.radius_search(pts, pts, radii, rs, rs)
    b = ops.radius_search(pts, pts, radii, rs, rs)
    assert torch.equal(a[0], b.neighbors_index)


@pytest.mark.gpu
def test_sparse_conv_autograd_through_registered_op(cuda):
    from o3dml_amd import layers, sparse_conv as sc
    g = torch.Generator().manual_seed(0)
    pos = torch.unique(torch.randint(0, 12, (600, 3), generator=g), dim=0).float().add(0.5).to(cuda)
    conv = layers.SparseConv(8, 16, [3, 3, 3], use_bias=False).to(cuda)
    conv.lattice_rulebook = False
    nb, kidx = conv._rulebook(pos, pos, 1.0, None, False, 1.0)
    x = torch.randn((pos.shape[0], 8), device=cuda, requires_grad=True)
    w = conv.kernel.detach().clone().requires_grad_(True)
    out = torch.ops.open3d.sparse_conv(w, x, None, nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
    go = torch.randn_like(out)
    gw, gx = torch.autograd.grad(out, (w, x), go)
    x2 = x.detach().clone().requires_grad_(True)
    w2 = w.detach().clone().requires_grad_(True)
    out2 = sc.sparse_conv(w2, x2, None, nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
    gw2, gx2 = torch.autograd.grad(out2, (w2, x2), go)
    assert torch.equal(out, out2)
    assert torch.equal(gw, gw2) and torch.equal(gx, gx2)
    # transpose: the adjoint, gradients through the registered op as well
    outT = torch.ops.open3d.sparse_conv_transpose(w, None, x, nb.neighbors_index, None, nb.neighbors_row_splits,
                                                  nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
    gwT, gxT = torch.autograd.grad(outT, (w, x), go)
    outT2 = sc.sparse_conv_transpose(w2, None, x2, nb.neighbors_index, None, nb.neighbors_row_splits,
                                     nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
    gwT2, gxT2 = torch.autograd.grad(outT2, (w2, x2), go)
    assert torch.equal(outT, outT2) and torch.equal(gwT, gwT2) and torch.equal(gxT, gxT2)


@pytest.mark.gpu
def test_three_interpolate_autograd(cuda):
    from o3dml_amd import ops
    feats = torch.randn((2, 6, 50), device=cuda, requires_grad=True)
    q = torch.rand((2, 80, 3), device=cuda)
    d = torch.rand((2, 50, 3), device=cuda)
    _, idx = ops.three_nn(q, d)
    w = torch.rand((2, 80, 3), device=cuda)
    out = torch.ops.open3d.three_interpolate(feats, idx, w)
    go = torch.randn_like(out)
    (gf,) = torch.autograd.grad(out, (feats,), go)
    ref = ops.three_interpolate_grad(go, idx, w, 50)
    assert torch.allclose(gf, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_registered_sparse_conv_backward_duplicate_kernel_indices(cuda):
    """Off-lattice positions (several neighbours of one output share a kernel
    index): the registered op's backward splits the pairs like the forward
    (sparse_conv._layered_grads) and equals sc.sparse_conv's gradients."""
    from o3dml_amd import layers, sparse_conv as sc
    rng = np.random.default_rng(5)
    pos = torch.from_numpy((rng.random((900, 3)) * 10).astype(np.float32)).to(cuda)
    conv = layers.SparseConv(8, 16, [3, 3, 3], use_bias=False).to(cuda)
    conv.lattice_rulebook = False
    nb, kidx = conv._rulebook(pos, pos, 1.0, None, False, 1.0)
    rs = nb.neighbors_row_splits.cpu()
    o = torch.repeat_interleave(torch.arange(rs.shape[0] - 1), rs[1:] - rs[:-1])
    assert torch.unique(o * 27 + kidx.long().cpu()).numel() < kidx.numel()  # duplicates present
    for normalize in (False, True):
        x = torch.randn((pos.shape[0], 8), device=cuda, requires_grad=True)
        w = conv.kernel.detach().clone().requires_grad_(True)
        out = torch.ops.open3d.sparse_conv(w, x, None, nb.neighbors_index, kidx, None, nb.neighbors_row_splits,
                                           normalize)
        go = torch.randn_like(out)
        gw, gx = torch.autograd.grad(out, (w, x), go)
        x2 = x.detach().clone().requires_grad_(True)
        w2 = w.detach().clone().requires_grad_(True)
        out2 = sc.sparse_conv(w2, x2, None, nb.neighbors_index, kidx, None, nb.neighbors_row_splits, normalize)
        gw2, gx2 = torch.autograd.grad(out2, (w2, x2), go)
        assert torch.equal(out, out2)
        assert torch.allclose(gw, gw2, rtol=1e-5, atol=1e-5) and torch.allclose(gx, gx2, rtol=1e-5, atol=1e-5)
        outT = torch.ops.open3d.sparse_conv_transpose(w, None, x, nb.neighbors_index, None, nb.neighbors_row_splits,
                                                      nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
        gwT, gxT = torch.autograd.grad(outT, (w, x), go)
        assert torch.isfinite(gwT).all() and torch.isfinite(gxT).all()


@pytest.mark.gpu
def test_transpose_importance_sum_needs_pair_importance(cuda):
    """sparse_conv_transpose(normalize=True) divides by the importance sum only
    when per-pair importances are given (Open3D's NEIGHBOR_IMPORTANCE †);
    without them by the neighbour count, whatever sum is passed (float64
    restatement)."""
    from o3dml_amd import layers, sparse_conv as sc
    g = torch.Generator().manual_seed(3)
    pos = torch.unique(torch.randint(0, 10, (500, 3), generator=g), dim=0).float().add(0.5).to(cuda)
    conv = layers.SparseConv(4, 6, [3, 3, 3], use_bias=False).to(cuda)
    conv.lattice_rulebook = False
    nb, kidx = conv._rulebook(pos, pos, 1.0, None, False, 1.0)
    n = pos.shape[0]
    x = torch.randn((n, 4), device=cuda)
    W = conv.kernel.detach()
    idx = nb.neighbors_index.long().cpu()
    rs = nb.neighbors_row_splits.cpu()
    o = torch.repeat_interleave(torch.arange(n), rs[1:] - rs[:-1])
    bogus_sum = torch.full((n,), 7.0, device=cuda)
    pair_imp = torch.rand(idx.numel(), device=cuda) + 0.5
    inp_sum = torch.zeros(n, dtype=torch.float64).index_add_(0, idx, pair_imp.double().cpu())
    cnt = torch.bincount(idx, minlength=n).double()
    W64 = W.double().cpu().reshape(27, 4, 6)
    x64 = x.double().cpu()
    for imp, den in ((None, cnt), (pair_imp, inp_sum)):
        s = bogus_sum if imp is None else inp_sum.float().to(cuda)
        out = sc.sparse_conv_transpose(W, None, x, idx.to(cuda).int(), s, rs, nb.neighbors_index, kidx, imp,
                                       nb.neighbors_row_splits, normalize=True)
        contrib = torch.einsum("pc,pcd->pd", x64[idx] / den[idx][:, None], W64[kidx.long().cpu()])
        if imp is not None:
            contrib = contrib * imp.double().cpu()[:, None]
        ref = torch.zeros((n, 6), dtype=torch.float64).index_add_(0, o, contrib)
        err = (out.double().cpu() - ref).abs().max() / ref.abs().max()
        assert err <= 1e-4, err


@pytest.mark.gpu
def test_ops_leave_current_device_unchanged(cuda):
    """An op on tensors of another GPU runs there under a restoring guard: the
    caller's current device is the same afterwards (needs 2 GPUs)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    from o3dml_amd import ops
    torch.cuda.set_device(0)
    pts = torch.rand((2000, 3), device="cuda:1")
    res = ops.fixed_radius_search(pts, pts, 0.1)
    assert res.neighbors_index.device == pts.device
    assert torch.cuda.current_device() == 0
