"""GPU parity for kNN, voxelize, grid subsampling and the PointNet++ ops vs the
C oracle: bit-exact for indices / ids / counts and for the float outputs whose
arithmetic order is shared (barycentres, interpolation); three_interpolate_grad
uses fp32 atomics -> rtol 1e-5 against the oracle's double accumulation."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _cloud(n, seed=0, scale=1.0, offset=0.0):
    return (np.random.default_rng(seed).random((n, 3), dtype=np.float32) * scale + offset).astype(np.float32)


# ------------------------------------------------------------------ kNN
@pytest.mark.parametrize("k", [1, 3, 16, 32, 64])
def test_knn_self(cuda, k):
    from o3dml_amd import ops
    pts = _cloud(6000, k)
    t = torch.from_numpy(pts).to(cuda)
    r = ops.knn_search(t, t, k, return_distances=True)
    oi, ors, od = O.knn_search(pts, pts, k, return_distances=True)
    assert np.array_equal(r.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(r.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(r.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("metric", ["L1", "Linf"])
def test_knn_metrics_ignore_batched(cuda, metric):
    from o3dml_amd import ops
    pts = _cloud(5000, 11, 3.0, -1.0)
    pts[10] = pts[20]
    qry = np.concatenate([_cloud(700, 12, 4.0, -1.5), pts[:300]])  # includes far-away queries
    prs = np.array([0, 2000, 5000], np.int64)
    qrs = np.array([0, 400, 1000], np.int64)
    r = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), 8, torch.from_numpy(prs),
                       torch.from_numpy(qrs), metric=metric, ignore_query_point=True, return_distances=True,
                       index_dtype=torch.int64)
    oi, ors, od = O.knn_search(pts, qry, 8, prs, qrs, metric=metric, ignore_query_point=True,
                               return_distances=True, index_dtype=np.int64)
    assert np.array_equal(r.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(r.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(r.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("k", [1, 16])
def test_knn_lidar_like_batched(cuda, k):
    """Surface data with a strongly varying density (a 64-beam scan: dense
    near the sensor, sparse far away) and RandLA-style nested levels batched
    in one call; bit-exact vs the oracle."""
    import bench
    pts, _ = bench.make_scan(3)
    lv = [pts[:20000], pts[:5000], pts[:1250]]
    cat = np.concatenate(lv)
    rs = np.array([0, 20000, 25000, 26250], np.int64)
    t = torch.from_numpy(cat).to(cuda)
    r = ops_knn(t, t, k, rs)
    oi, ors, od = O.knn_search(cat, cat, k, rs, rs, return_distances=True)
    assert np.array_equal(r.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(r.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(r.neighbors_distance.cpu().numpy(), od)


def ops_knn(p, q, k, rs):
    from o3dml_amd import ops
    return ops.knn_search(p, q, k, torch.from_numpy(rs), torch.from_numpy(rs), return_distances=True)


def test_knn_small_batches_and_duplicates(cuda):
    from o3dml_amd import ops
    pts = np.repeat(_cloud(50, 3), 4, axis=0)  # exact duplicates -> ties broken by index
    prs = np.array([0, 5, 5, 200], np.int64)  # batch with fewer points than k, an empty batch
    r = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(pts).to(cuda), 16,
                       torch.from_numpy(prs), torch.from_numpy(prs), return_distances=True)
    oi, ors, od = O.knn_search(pts, pts, 16, prs, prs, return_distances=True)
    assert np.array_equal(r.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(r.neighbors_index.cpu().numpy(), oi)


def test_knn_large_k_patch_crop(cuda):
    """k > 64: the sampler's single-centre crop (semseg_spatially_regular.py:94-95)."""
    from o3dml_amd import ops
    pts = _cloud(20000, 4, 10.0)
    ctr = pts[123:124].copy()
    r = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(ctr).to(cuda), 4096,
                       return_distances=True)
    oi, ors, od = O.knn_search(pts, ctr, 4096, return_distances=True)
    assert np.array_equal(r.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(r.neighbors_distance.cpu().numpy(), od)


def test_core_nns_knn(cuda):
    """open3d.core.nns path used by DataProcessing.knn_search (dataprocessing.py:99-101)."""
    import open3d.core as o3c
    sup = _cloud(3000, 5)
    qry = _cloud(2000, 6)
    nns = o3c.nns.NearestNeighborSearch(o3c.Tensor.from_numpy(sup))
    nns.knn_index()
    idx, dist = nns.knn_search(o3c.Tensor.from_numpy(qry), 16)
    oi, _, od = O.knn_search(sup, qry, 16, return_distances=True)
    assert idx.numpy().dtype == np.int64 and idx.numpy().shape == (2000, 16)
    assert np.array_equal(idx.numpy().reshape(-1), oi)
    assert np.array_equal(dist.numpy().reshape(-1), od)


# ------------------------------------------------------------------ voxelize
def test_voxelize_pointpillars_shape(cuda):
    from o3dml_amd import ops
    rng = np.random.default_rng(8)
    pts = np.stack([rng.uniform(-2, 71, 30000), rng.uniform(-41, 41, 30000), rng.uniform(-3.5, 1.5, 30000)],
                   1).astype(np.float32)
    rs = np.array([0, 12000, 30000], np.int64)
    vs, mn, mx = [0.16, 0.16, 4.0], [0, -39.68, -3], [69.12, 39.68, 1]
    for caps in [(2**63 - 1, 2**63 - 1), (32, 16000), (3, 500)]:
        r = ops.voxelize(torch.from_numpy(pts).to(cuda), torch.from_numpy(rs).to(cuda), torch.tensor(vs),
                         torch.tensor(mn), torch.tensor(mx), *caps)
        o = O.voxelize(pts, rs, vs, mn, mx, *caps)
        assert np.array_equal(r.voxel_coords.cpu().numpy(), o[0])
        assert np.array_equal(r.voxel_point_indices.cpu().numpy(), o[1])
        assert np.array_equal(r.voxel_point_row_splits.cpu().numpy(), o[2])
        assert np.array_equal(r.voxel_batch_splits.cpu().numpy(), o[3])


def test_voxelize_sparseconv_input_layer(cuda):
    """InputLayer (sparseconvnet.py:293-298): vs=1, range [0, 40960)^3."""
    from o3dml_amd import ops
    pts = (np.random.default_rng(9).random((20000, 3)) * 200).astype(np.float32)
    r = ops.voxelize(torch.from_numpy(pts).to(cuda), torch.LongTensor([0, 20000]).to(cuda),
                     torch.Tensor([1, 1, 1]), torch.Tensor([0, 0, 0]), torch.Tensor([40960] * 3))
    o = O.voxelize(pts, [0, 20000], [1, 1, 1], [0, 0, 0], [40960] * 3)
    for a, b in zip(r, o):
        assert np.array_equal(a.cpu().numpy(), b)


# ------------------------------------------------------------------ grid subsample
def test_contrib_subsample_randla(cuda):
    from open3d.ml.contrib import subsample
    rng = np.random.default_rng(10)
    pts = (rng.random((40000, 3)) * [40, 40, 3] - [20, 20, 1.7]).astype(np.float32)
    lab = rng.integers(0, 19, 40000).astype(np.int32)
    feat = rng.random((40000, 4)).astype(np.float32)
    sp, sf, sl = subsample(pts, features=feat, classes=lab, sampleDl=0.06)
    op, of, ol = O.subsample(pts, features=feat, classes=lab, sampleDl=0.06)
    assert np.array_equal(sp, op) and np.array_equal(sf, of) and np.array_equal(sl, ol)
    only = subsample(pts, sampleDl=0.1)
    assert np.array_equal(only, O.subsample(pts, sampleDl=0.1))


def test_contrib_subsample_batch_maxp(cuda):
    from open3d.ml.contrib import subsample_batch
    rng = np.random.default_rng(11)
    lens = np.array([5000, 0, 12000, 3000], np.int32)
    pts = (rng.standard_normal((lens.sum(), 3)) * 2).astype(np.float32)
    for max_p in [0, 700]:
        a = subsample_batch(pts, lens, sampleDl=0.2, max_p=max_p)
        b = O.subsample_batch(pts, lens, sampleDl=0.2, max_p=max_p)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


# ------------------------------------------------------------------ PointNet++
@pytest.mark.parametrize("n,m", [(1000, 100), (16384, 4096), (40000, 64)])
def test_fps(cuda, n, m):
    from o3dml_amd import ops
    pts = np.random.default_rng(n).random((2, n, 3), dtype=np.float32)
    r = ops.furthest_point_sampling(torch.from_numpy(pts).to(cuda), m)
    assert np.array_equal(r.cpu().numpy(), O.furthest_point_sampling(pts, m))


def test_ball_query_three_nn_interp(cuda):
    from o3dml_amd import ops
    rng = np.random.default_rng(12)
    xyz = rng.random((2, 3000, 3), dtype=np.float32)
    ctr = rng.random((2, 500, 3), dtype=np.float32)
    ctr[0, 0] = 5.0  # no neighbour -> zeros
    bq = ops.ball_query(torch.from_numpy(xyz).to(cuda), torch.from_numpy(ctr).to(cuda), 0.1, 16)
    assert np.array_equal(bq.cpu().numpy(), O.ball_query(xyz, ctr, 0.1, 16))
    d, i = ops.three_nn(torch.from_numpy(ctr).to(cuda), torch.from_numpy(xyz).to(cuda))
    od, oi = O.three_nn(ctr, xyz)
    assert np.array_equal(i.cpu().numpy(), oi) and np.array_equal(d.cpu().numpy(), od)
    w = rng.random((2, 500, 3)).astype(np.float32)
    f = rng.standard_normal((2, 8, 3000)).astype(np.float32)
    out = ops.three_interpolate(torch.from_numpy(f).to(cuda), i, torch.from_numpy(w).to(cuda))
    assert np.array_equal(out.cpu().numpy(), O.three_interpolate(f, oi, w))
    g = rng.standard_normal((2, 8, 500)).astype(np.float32)
    gf = ops.three_interpolate_grad(torch.from_numpy(g).to(cuda), i, torch.from_numpy(w).to(cuda), 3000)
    np.testing.assert_allclose(gf.cpu().numpy(), O.three_interpolate_grad(g, oi, w, 3000), rtol=1e-5, atol=1e-6)
