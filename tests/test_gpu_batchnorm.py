"""csrc/bn.hip (o3dml_amd.batchnorm.bn_act) vs torch's nn.BatchNorm1d +
nn.LeakyReLU in fp32 (KPFCNN BatchNormBlock, ml3d/torch/models/kpconv.py:
1213-1295): outputs, running statistics, num_batches_tracked, input / weight /
bias gradients, train and eval, packed (C <= 256) and channel-block (C > 256)
layouts.  Tolerances: fp32 rounding of a double-accumulated reduction vs
torch's fp32 Welford (rtol 1e-5 on y, 1e-4 on gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,c", [(2, 16), (1000, 64), (40000, 128), (777, 100), (3000, 300), (2048, 1024)])
@pytest.mark.parametrize("slope", [None, 0.1])
def test_bn_act_train_matches_torch(cuda, n, c, slope):
    from o3dml_amd.batchnorm import bn_act
    g = torch.Generator().manual_seed(n + c)
    x0 = (torch.randn(n, c, generator=g) * 3 + 1.5).to(cuda)
    ref = torch.nn.BatchNorm1d(c, momentum=0.02).to(cuda)
    ours = torch.nn.BatchNorm1d(c, momentum=0.02).to(cuda)
    with torch.no_grad():
        for m in (ref, ours):
            m.weight.copy_(torch.linspace(0.5, 1.5, c))
            m.bias.copy_(torch.linspace(-0.2, 0.3, c))
            m.running_mean.copy_(torch.linspace(0, 1, c))
            m.running_var.copy_(torch.linspace(1, 2, c))
    xr = x0.clone().requires_grad_()
    xo = x0.clone().requires_grad_()
    yr = ref(xr)
    if slope is not None:
        yr = torch.nn.functional.leaky_relu(yr, slope)
    yo = bn_act(xo, ours, slope)
    torch.testing.assert_close(yo, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ours.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ours.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(ours.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    gy = torch.randn(n, c, generator=g).to(cuda)
    yr.backward(gy)
    yo.backward(gy)
    torch.testing.assert_close(xo.grad, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ours.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("c", [64, 512])
def test_bn_act_eval_matches_torch(cuda, c):
    from o3dml_amd.batchnorm import bn_act
    g = torch.Generator().manual_seed(c)
    ref = torch.nn.BatchNorm1d(c).to(cuda)
    with torch.no_grad():
        ref.running_mean.copy_(torch.randn(c, generator=g))
        ref.running_var.copy_(torch.rand(c, generator=g) + 0.5)
        ref.weight.copy_(torch.randn(c, generator=g))
    ref.eval()
    x = torch.randn(500, c, generator=g).to(cuda).requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    yr = torch.nn.functional.leaky_relu(ref(x), 0.1)
    yo = bn_act(x2, ref, 0.1)
    torch.testing.assert_close(yo, yr, rtol=1e-5, atol=1e-6)
    gy = torch.randn(500, c, generator=g).to(cuda)
    yr.backward(gy)
    wr, br = ref.weight.grad.clone(), ref.bias.grad.clone()
    ref.weight.grad = ref.bias.grad = None
    yo.backward(gy)
    torch.testing.assert_close(x2.grad, x.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ref.weight.grad, wr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ref.bias.grad, br, rtol=1e-4, atol=1e-4)
    assert int(ref.num_batches_tracked) == 0


def test_bn_act_deterministic_and_graph_capturable(cuda):
    """Bitwise run to run (block-order sums), and a captured forward replays."""
    from o3dml_amd.batchnorm import bn_act
    x = torch.randn(40000, 128, device=cuda)
    bn = torch.nn.BatchNorm1d(128).to(cuda)
    a = bn_act(x, bn, 0.1)
    b = bn_act(x, bn, 0.1)
    assert torch.equal(a, b)
    bn.eval()
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        bn_act(x, bn, 0.1)
    torch.cuda.current_stream(cuda).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = bn_act(x, bn, 0.1)
    g.replay()
    torch.testing.assert_close(out, torch.nn.functional.leaky_relu(bn(x), 0.1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_sgemm_matches_torch(cuda, ta, tb):
    """o3dml_sgemm (rocBLAS, csrc/gemm.cpp) row-major with transposes."""
    from o3dml_amd._util import mm
    g = torch.Generator().manual_seed(int(ta) * 2 + int(tb))
    m, n, k = 1000, 48, 37
    a = torch.randn((k, m) if ta else (m, k), generator=g).to(cuda)
    b = torch.randn((n, k) if tb else (k, n), generator=g).to(cuda)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double()
    torch.testing.assert_close(mm(a, b, ta, tb).double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("k", [4096, 40000, 40001, 200000])
@pytest.mark.parametrize("ta,tb", [(True, False), (False, False), (False, True), (True, True)])
def test_sgemm_splitk_matches_torch(cuda, k, ta, tb):
    """Long-reduction GEMMs through the split-K path (equal parts + tail,
    slabs summed in order), every transpose: vs fp64, and bitwise run to run."""
    from o3dml_amd._util import mm
    g = torch.Generator().manual_seed(k + 2 * int(ta) + int(tb))
    m, n = 96, 40
    a = torch.randn((k, m) if ta else (m, k), generator=g).to(cuda)
    b = torch.randn((n, k) if tb else (k, n), generator=g).to(cuda)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double()
    got = mm(a, b, ta, tb)
    torch.testing.assert_close(got.double(), ref, rtol=1e-4, atol=1e-3 * k ** 0.5 / 100)
    assert torch.equal(got, mm(a, b, ta, tb))
