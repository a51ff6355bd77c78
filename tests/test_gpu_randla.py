"""RandLA-Net on the GPU: the fused HIP path (csrc/randla.hip + folded
BatchNorm GEMMs) against the reference logits (tests/golden/randla.npz,
fp32, tolerance 2e-4 abs on logits of magnitude ~2), the three kernels
against torch fp32 restatements, and the GPU inference pipeline."""
import numpy as np
import pytest
import torch

from test_randla import G, golden_inputs, golden_model

pytestmark = pytest.mark.gpu


def test_fused_forward_matches_reference(cuda):
    m = golden_model().to(cuda)
    with torch.no_grad():
        out = m(golden_inputs(lambda t: t.to(cuda)))[0].cpu().numpy()
    np.testing.assert_allclose(out, G["logits"], rtol=0, atol=2e-4)


def test_kernels_vs_torch(cuda):
    from o3dml_amd import randlanet as R
    g = torch.Generator().manual_seed(3)
    coords = torch.rand((500, 3), generator=g).to(cuda)
    nbr = torch.randint(0, 500, (500, 16), generator=g, dtype=torch.int32).to(cuda)
    rel = R.relative_encoding(coords, nbr)
    nc = coords[nbr.long()]
    ext = coords[:, None, :].expand(500, 16, 3)
    rp = ext - nc
    ref = torch.cat([torch.sqrt((rp * rp).sum(-1, keepdim=True)), rp, ext, nc], -1)
    torch.testing.assert_close(rel, ref, rtol=1e-6, atol=1e-6)
    x = torch.randn((500, 16, 24), generator=g).to(cuda)
    lg = torch.randn((500, 16, 24), generator=g).to(cuda)
    torch.testing.assert_close(R.attentive_pool(x, lg), (torch.softmax(lg, 1) * x).sum(1), rtol=1e-5, atol=1e-5)
    feat = torch.randn((500, 40), generator=g).to(cuda)
    idx = torch.randint(0, 500, (120, 16), generator=g, dtype=torch.int32).to(cuda)
    torch.testing.assert_close(R.gather_max(feat, idx), feat[idx.long()].max(1).values)
    b = torch.randn((120 * 16, 7), generator=g).to(cuda)
    assert torch.equal(R.concat_rows(feat, idx.reshape(-1), b, None), torch.cat([feat[idx.reshape(-1).long()], b], 1))
    up = torch.randint(0, 120 * 16, (500,), generator=g).to(cuda)
    assert torch.equal(R.concat_rows(feat, None, b, up), torch.cat([feat, b[up]], 1))


def test_inference_pipeline_covers_cloud(cuda):
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda)
    rng = np.random.default_rng(1)
    pts = np.stack([rng.uniform(-20, 20, 30000), rng.uniform(-20, 20, 30000), rng.uniform(-2, 2, 30000)], 1)
    pts = torch.from_numpy(pts.astype(np.float32)).to(cuda)
    inf = SemSegInference(m, seed=0)
    labels, probs = inf.run(pts)
    assert labels.shape == (30000,) and probs.shape == (30000, 19)
    assert inf.stats["patches"] >= 1
    assert torch.isfinite(probs).all() and (probs.sum(1) > 0).all()
    labels2, _ = SemSegInference(m, seed=0).run(pts)
    assert torch.equal(labels, labels2)  # seeded -> reproducible patch sequence


@pytest.mark.parametrize("d_out", [16, 64, 128, 256])
def test_fused_pooling_widths_vs_torch(cuda, d_out):
    """Fused LSE + attentive pooling (VALU kernel below 64 channels, MFMA kernel
    from 64 up) against the module's own torch path, eval mode, odd point count
    (the MFMA kernel's half-filled last pair of points)."""
    from o3dml_amd.randlanet import LocalFeatureAggregation
    torch.manual_seed(d_out)
    n = 301
    m = LocalFeatureAggregation(d_out // 2, d_out, 16).to(cuda).eval()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.2, 0.2)
            mod.running_var.uniform_(0.5, 1.5)
    coords = torch.rand((n, 3), device=cuda) * 4.0
    feat = torch.randn((n, d_out // 2), device=cuda)
    nbr = torch.randint(0, n, (n, 16), device=cuda, dtype=torch.int32)
    with torch.no_grad():
        fused = m(coords, feat, nbr)
    with torch.enable_grad():
        ref = m(coords, feat, nbr).detach()
    torch.testing.assert_close(fused, ref, rtol=1e-4, atol=1e-4)


def test_inference_graph_replay_matches_eager(cuda):
    """The patch network replayed as a HIP graph gives the eager path's result."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda)
    rng = np.random.default_rng(2)
    pts = np.stack([rng.uniform(-20, 20, 20000), rng.uniform(-20, 20, 20000), rng.uniform(-2, 2, 20000)], 1)
    pts = torch.from_numpy(pts.astype(np.float32)).to(cuda)
    lg, pg = SemSegInference(m, seed=0, use_graph=True, probs_dtype=torch.float32).run(pts)
    le, pe = SemSegInference(m, seed=0, use_graph=False, probs_dtype=torch.float32).run(pts)
    torch.testing.assert_close(pg, pe, rtol=0, atol=1e-6)
    assert torch.equal(lg, le)


def test_dense_act_vs_torch(cuda):
    """csrc/dense.hip: act([a1 | a2[idx]] @ W^T + b) against torch fp32, for the
    tile shapes the model uses (outputs 8 .. 512 wide, 1 .. 45,056 rows)."""
    from o3dml_amd.randlanet import dense_act
    g = torch.Generator().manual_seed(5)
    for n, k1, k2, m, slope, idx in ((45056, 3, 0, 8, 0.2, False), (11264, 32, 32, 128, 0.01, False),
                                     (704, 256, 512, 256, 0.2, True), (1, 16, 0, 19, None, False),
                                     (2816, 128, 128, 64, 0.2, True)):
        a1 = torch.randn((n, k1), generator=g).to(cuda)
        a2 = torch.randn((max(n // 4, 1), k2), generator=g).to(cuda) if k2 else None
        ix = torch.randint(0, max(n // 4, 1), (n,), generator=g).to(cuda) if (k2 and idx) else None
        if k2 and not idx:
            a2 = torch.randn((n, k2), generator=g).to(cuda)
        w = (torch.randn((m, k1 + k2), generator=g) / (k1 + k2) ** 0.5).to(cuda)
        b = torch.randn(m, generator=g).to(cuda)
        got = dense_act(a1, w, b, slope, a2=a2, a2_index=ix)
        x = a1 if a2 is None else torch.cat([a1, a2[ix] if ix is not None else a2], 1)
        ref = x.double() @ w.double().t() + b.double()
        if slope is not None:
            ref = torch.nn.functional.leaky_relu(ref, slope)
        torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=1e-5)


def test_up_from_knn_equals_second_search(cuda):
    """Up-sampling indices from the k=16 lists == knn_search(level i+1, level i, 1)
    on the four nested RandLA levels of a scan patch (incl. the brute-force
    fallback for points with no prefix point among their 16)."""
    import bench
    from o3dml_amd import ops
    from o3dml_amd.randlanet import up_from_knn
    pts, _ = bench.make_scan(2)
    pc = torch.from_numpy(pts[:45056]).to(cuda)
    sizes = [45056, 11264, 2816, 704, 176]
    cat = torch.cat([pc[:s] for s in sizes[:4]]).contiguous()
    rs = np.concatenate([[0], np.cumsum(sizes[:4])]).astype(np.int64)
    srs = np.concatenate([[0], np.cumsum(sizes[1:])]).astype(np.int64)
    nb = ops.knn_search(cat, cat, 16, rs, rs).neighbors_index.view(-1, 16)
    nb0 = nb.clone()
    got = up_from_knn(nb, cat, rs, np.asarray(sizes[1:], np.int64), srs)
    sup = torch.cat([pc[:s] for s in sizes[1:]]).contiguous()
    ref = ops.knn_search(sup, cat, 1, srs, rs).neighbors_index.long()
    lvl = torch.repeat_interleave(torch.arange(4, device=cuda), torch.tensor(sizes[:4], device=cuda))
    assert torch.equal(got, ref - torch.from_numpy(srs[:4]).to(cuda)[lvl])  # relative to level i+1
    assert torch.equal(nb.long(), nb0.long() - torch.from_numpy(rs[:4]).to(cuda)[lvl][:, None])  # rebased
    # the fallback path really ran: points whose 16 lie outside the prefix
    assert ((nb[:45056] >= 11264).all(1)).sum() > 0


def test_patch_update_matches_reference_arithmetic(cuda):
    """o3dml_randla_patch_update / _possibility_min against the reference's
    numpy arithmetic (semseg_spatially_regular.py:100-106): possibilities
    bit-exact, first argmin, recentred patch within 1e-5."""
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle
    rng = np.random.default_rng(4)
    sub = rng.uniform(-40, 40, (20000, 3)).astype(np.float32)
    poss = rng.random(20000) * 1e-3
    poss[[17, 900]] = poss.min() / 2  # a tie: the first index wins
    lib = _lib.load()
    sub_t, poss_t = torch.from_numpy(sub).to(cuda), torch.from_numpy(poss).to(cuda)
    arg = torch.empty(1, dtype=torch.int64, device=cuda)
    center = torch.empty(3, device=cuda)
    host_min = torch.empty(1, dtype=torch.float64, pin_memory=True)
    mws = torch.empty(lib.o3dml_randla_possibility_min_workspace_size(), dtype=torch.uint8, device=cuda)
    _lib.call("o3dml_randla_possibility_min", ptr(poss_t), 20000, ptr(sub_t), ptr(arg), ptr(center),
              host_min.data_ptr(), ptr(mws), mws.numel(), stream_handle(cuda))
    torch.cuda.synchronize()
    assert int(arg) == int(np.argmin(poss)) == 17 and float(host_min[0]) == poss.min()
    assert np.array_equal(center.cpu().numpy(), sub[17])
    idxs = rng.permutation(20000)[:4096]
    pc = torch.empty((4096, 3), device=cuda)
    ws = torch.empty(lib.o3dml_randla_patch_workspace_size(4096), dtype=torch.uint8, device=cuda)
    idx_t = torch.from_numpy(idxs.astype(np.int64)).to(cuda)
    _lib.call("o3dml_randla_patch_update", ptr(sub_t), ptr(idx_t), 4096, ptr(center), None, ptr(poss_t), ptr(pc),
              ptr(ws), ws.numel(), stream_handle(cuda))
    ref_pc = sub[idxs]
    dists = np.sum(np.square((ref_pc - sub[17:18]).astype(np.float32)), axis=1)
    delta = np.square(1 - dists / np.max(dists))
    ref_poss = poss.copy()
    ref_poss[idxs] += delta
    assert np.array_equal(poss_t.cpu().numpy(), ref_poss)
    rc = ref_pc.copy()
    rc[:, [0, 1]] = rc[:, [0, 1]] - rc.mean(0)[[0, 1]]
    np.testing.assert_allclose(pc.cpu().numpy(), rc, rtol=0, atol=1e-5)


def test_random_permute_is_a_permutation(cuda):
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle
    for n in (1, 2, 45056, 65537):
        src = torch.arange(n, device=cuda) * 3
        dst = torch.empty_like(src)
        _lib.call("o3dml_random_permute", ptr(src), n, 12345, ptr(dst), stream_handle(cuda))
        assert torch.equal(torch.sort(dst).values, src)
        if n > 1000:
            assert (dst != src).float().mean() > 0.99  # actually shuffled
            d2 = torch.empty_like(src)
            _lib.call("o3dml_random_permute", ptr(src), n, 12345, ptr(d2), stream_handle(cuda))
            assert torch.equal(dst, d2)  # keyed: deterministic


def test_update_probs_matches_reference_float16(cuda):
    """o3dml_randla_update_probs == the reference's numpy float16 EMA
    (randlanet.py:462: f16 store, Python scalars) bit for bit."""
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle
    rng = np.random.default_rng(9)
    tp = rng.random((3000, 19)).astype(np.float16)
    probs = rng.random((1000, 19)).astype(np.float32)
    idxs = rng.permutation(3000)[:1000]
    ref = tp.copy()
    ref[idxs] = 0.95 * ref[idxs] + (1 - 0.95) * probs
    t = torch.from_numpy(tp).to(cuda)
    p_d = torch.from_numpy(probs).to(cuda)  # named: a temporary could be recycled before the launch
    i_d = torch.from_numpy(idxs.astype(np.int64)).to(cuda)
    _lib.call("o3dml_randla_update_probs", ptr(p_d), ptr(i_d), None, 1000, 19, 0.95, 1, ptr(t), stream_handle(cuda))
    assert np.array_equal(t.cpu().numpy(), ref)


def test_dense_fused_split_reduce_bitwise(cuda, tmp_path):
    """The optional split-K finish in the last-arriving block of each tile
    (O3DML_DENSE_FUSED_REDUCE=1, per-tile counters) against the default
    two-launch form: same split order, so bit-identical (child processes:
    the switch is read once)."""
    import os
    import subprocess
    import sys
    code = ("import torch,sys; sys.path.insert(0,'open3d-ml_amd'); from o3dml_amd.randlanet import dense_act;"
            "torch.manual_seed(0); r=[]\n"
            "for n,k,m in ((704,768,512),(2816,256,128),(176,512,512),(45056,8,16)):\n"
            "  a=torch.randn((n,k),device='cuda'); w=torch.randn((m,k),device='cuda')/k**0.5; b=torch.randn(m,device='cuda')\n"
            "  r.append(dense_act(a,w,b,0.2).cpu())\n"
            "torch.save(r, sys.argv[1])")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for flag in ("1", "0"):
        path = str(tmp_path / f"dense_reduce_{flag}.pt")
        env = dict(os.environ, O3DML_DENSE_FUSED_REDUCE=flag)
        subprocess.run([sys.executable, "-c", code, path], check=True, env=env, cwd=root, timeout=120)
        outs.append(torch.load(path, weights_only=True))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_patch_step_equals_ops(cuda):
    """The capturable patch step (SemSegInference._patch_step, direct ABI
    calls over padded static buffers) produces exactly what the op-level
    pipeline would: the crop = the set of ops.knn_search(sub, centre,
    num_points) (L2) in index order (radix selection, o3dml_knn_select), the
    shuffled indices a permutation of it, the
    per-level k-lists = ops.knn_search on the levels, the up-sampling ids =
    a second 1-NN search, and the possibility update of the crop."""
    from o3dml_amd import ops
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda)
    rng = np.random.default_rng(3)
    pts = np.stack([rng.uniform(-20, 20, 30000), rng.uniform(-20, 20, 30000), rng.uniform(-2, 2, 30000)], 1)
    pts = torch.from_numpy(pts.astype(np.float32)).to(cuda)
    inf = SemSegInference(m, seed=0, use_graph=False)
    sub, _ = inf.preprocess(pts)
    n = sub.shape[0]
    step = inf._patch_step(n)
    p0 = torch.rand(n, generator=torch.Generator(device=cuda).manual_seed(5), device=cuda, dtype=torch.float64)
    step.begin(sub, p0, 123)
    center = step.center.clone()
    assert int(step.arg) == int(torch.argmin(p0))
    with torch.no_grad():
        step.step()
    crop = ops.knn_search(sub, center.view(1, 3), 4096, index_dtype=torch.int64).neighbors_index
    assert torch.equal(step.crop, torch.sort(crop).values)
    assert torch.equal(torch.sort(step.idxs).values, torch.sort(crop).values)
    sizes, rs, _ = step.plan
    cat = step.cat
    ref = ops.knn_search(cat, cat, 16, rs, rs).neighbors_index.view(-1, 16).long()
    base = torch.repeat_interleave(torch.from_numpy(rs[:-1]).to(cuda), torch.from_numpy(np.diff(rs)).to(cuda))
    assert torch.equal(step.nb.long(), ref - base[:, None])  # rewritten level-relative by up_from_knn
    for i in range(len(sizes) - 1):
        lvl, nxt = cat[rs[i]:rs[i + 1]], cat[rs[i]:rs[i] + sizes[i + 1]]
        up = ops.knn_search(nxt, lvl, 1, index_dtype=torch.int64).neighbors_index
        assert torch.equal(step.up[rs[i]:rs[i + 1]], up)
    grew = step.poss[:n][crop] > p0[crop]  # delta = (1 - d / d_max)^2: 0 only at the farthest point
    assert torch.all(step.poss[:n][crop] >= p0[crop]) and int(grew.sum()) >= crop.numel() - 1
    untouched = torch.ones(n, dtype=torch.bool, device=cuda)
    untouched[crop] = False
    assert torch.equal(step.poss[:n][untouched], p0[untouched])


def test_patch_graph_survives_frames_and_drops_with_weights(cuda):
    """The captured patch step holds raw pointers to the folded eval weights:
    a second frame on the same model reuses the graph AND the folded weights
    (run() calls eval() per frame, which must not free them), its result equals
    the eager launches on the same frame; a mode switch or a state_dict load
    drops the graphs with the weights they point at."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda).eval()
    rng = np.random.default_rng(4)

    def cloud():
        p = np.stack([rng.uniform(-20, 20, 20000), rng.uniform(-20, 20, 20000), rng.uniform(-2, 2, 20000)], 1)
        return torch.from_numpy(p.astype(np.float32)).to(cuda)

    a, b = cloud(), cloud()
    SemSegInference(m, seed=1, use_graph=True, probs_dtype=torch.float32).run(a)
    steps = m.__dict__["_o3dml_patch_step"]
    assert len(steps) == 1
    step = next(iter(steps.values()))
    folded = m.encoder[0].mlp1.folded()[0]
    lg, pg = SemSegInference(m, seed=2, use_graph=True, probs_dtype=torch.float32).run(b)
    assert step in m.__dict__["_o3dml_patch_step"].values() and step.graph is not None
    assert m.encoder[0].mlp1.folded()[0] is folded
    le, pe = SemSegInference(m, seed=2, use_graph=False, probs_dtype=torch.float32).run(b)
    torch.testing.assert_close(pg, pe, rtol=0, atol=1e-6)
    assert torch.equal(lg, le)
    m.train()
    assert "_o3dml_patch_step" not in m.__dict__
    m.eval()
    SemSegInference(m, seed=1, use_graph=True).run(a)
    m.load_state_dict(m.state_dict())
    assert "_o3dml_patch_step" not in m.__dict__


def test_knn_select_in_graph_equals_eager(cuda):
    """o3dml_knn_select (zero + three histogram + count + write launches)
    captured in a HIP graph and replayed for a moving centre gives the eager
    call's set."""
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle
    lib = _lib.load()
    rng = np.random.default_rng(6)
    n, k = 98304, 45056
    pts = torch.from_numpy(rng.uniform(-30, 30, (n, 3)).astype(np.float32)).to(cuda)
    center = torch.zeros(3, dtype=torch.float32, device=cuda)
    ws = torch.empty(lib.o3dml_knn_select_workspace_size(n), dtype=torch.uint8, device=cuda)
    out = torch.empty(k, dtype=torch.int64, device=cuda)

    def call():
        _lib.call("o3dml_knn_select", ptr(pts), n, ptr(center), k, 1, ptr(out), ptr(ws), ws.numel(),
                  stream_handle(cuda))

    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):
        call()
    torch.cuda.current_stream(cuda).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        call()
    for i in range(4):
        center.copy_(pts[i * 1000])
        g.replay()
        got = out.clone()
        call()
        assert torch.equal(got, out), i
        assert torch.all(got[1:] > got[:-1]), i  # a set, in index order
        d = ((pts - pts[i * 1000]) ** 2).sum(1)
        rest = torch.ones(n, dtype=torch.bool, device=cuda)
        rest[got] = False
        assert float(d[got].max()) <= float(d[rest].min()) * (1 + 1e-5), i


def test_patch_steps_kept_per_capacity(cuda):
    """Scans whose sub-clouds fall into different capacity classes keep one
    captured patch step each (up to _MAX_STEPS): alternating between them
    replays the existing graphs instead of re-capturing."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda).eval()
    rng = np.random.default_rng(7)

    def cloud(n):
        p = np.stack([rng.uniform(-20, 20, n), rng.uniform(-20, 20, n), rng.uniform(-2, 2, n)], 1)
        return torch.from_numpy(p.astype(np.float32)).to(cuda)

    small, large = cloud(20000), cloud(40000)
    SemSegInference(m, seed=1, use_graph=True).run(small)
    SemSegInference(m, seed=1, use_graph=True).run(large)
    steps = dict(m.__dict__["_o3dml_patch_step"])
    assert len(steps) == 2 and all(s.graph is not None for s in steps.values())
    SemSegInference(m, seed=2, use_graph=True).run(small)
    after = m.__dict__["_o3dml_patch_step"]
    assert set(after) == set(steps) and all(after[k] is steps[k] for k in steps)


def test_patch_step_eviction_recapture_and_empty_cache(cuda):
    """More sub-cloud capacity classes than _MAX_STEPS: steps are evicted
    (their graphs destroyed), an evicted class comes back and is re-captured,
    the caching allocator is emptied and churned between frames (VERDICT r4
    item 1: the r4fin1 fault ran right after a capacity-class switch that
    destroyed a graph and captured a new one).  Every graph frame equals the
    same frame issued eagerly through the same step buffers."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda).eval()
    rng = np.random.default_rng(11)

    def cloud(n):
        p = np.stack([rng.uniform(-20, 20, n), rng.uniform(-20, 20, n), rng.uniform(-2, 2, n)], 1)
        return torch.from_numpy(p.astype(np.float32)).to(cuda)

    # sub-clouds in five capacity classes (16,384-point granularity) > _MAX_STEPS = 4
    clouds = [cloud(n) for n in (8000, 24000, 40000, 56000, 72000)]
    assert SemSegInference._MAX_STEPS == 4
    caps, seen = set(), []
    for f, i in enumerate((0, 1, 2, 3, 4, 0, 4, 1, 0)):
        junk = [torch.empty(int(s), dtype=torch.uint8, device=cuda) for s in rng.integers(1 << 10, 1 << 24, 6)]
        del junk
        torch.cuda.empty_cache()
        lg, pg = SemSegInference(m, seed=f, use_graph=True, probs_dtype=torch.float32).run(clouds[i])
        torch.cuda.synchronize(cuda)
        steps = m.__dict__["_o3dml_patch_step"]
        assert len(steps) <= SemSegInference._MAX_STEPS
        key = next(reversed(steps))  # most recently used: this frame's class
        step = steps[key]
        assert step.graph is not None
        seen.append(step)
        caps.add(key[1])
        le, pe = SemSegInference(m, seed=f, use_graph=False, probs_dtype=torch.float32).run(clouds[i])
        torch.testing.assert_close(pg, pe, rtol=0, atol=1e-6)
        assert torch.equal(lg, le), f
    assert len(caps) == 5
    # class 0 was evicted by class 4 and re-captured (a new step object)
    assert seen[5] is not seen[0] and seen[8] is seen[5]


def test_folded_weights_follow_in_place_parameter_updates(cuda):
    """An in-place parameter update in eval mode (an optimizer step, copy_)
    bumps the tensor's version counter: the next frame drops the folded eval
    weights and the graphs captured on them and rebuilds both;
    .to() (Module._apply) drops them too."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    m = RandLANet(num_points=4096).to(cuda).eval()
    rng = np.random.default_rng(12)
    p = np.stack([rng.uniform(-20, 20, 20000), rng.uniform(-20, 20, 20000), rng.uniform(-2, 2, 20000)], 1)
    pts = torch.from_numpy(p.astype(np.float32)).to(cuda)
    SemSegInference(m, seed=1).run(pts)
    step = next(iter(m.__dict__["_o3dml_patch_step"].values()))
    with torch.no_grad():
        m.fc1[-1].conv.bias[3] += 100.0  # class 3 dominates every point
    lg, _ = SemSegInference(m, seed=1).run(pts)
    assert bool((lg == 3).all())
    assert next(iter(m.__dict__["_o3dml_patch_step"].values())) is not step  # re-captured
    le, _ = SemSegInference(m, seed=1, use_graph=False).run(pts)
    assert torch.equal(lg, le)
    m.to(cuda)
    assert "_o3dml_patch_step" not in m.__dict__
