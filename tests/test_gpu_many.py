"""GPU parity of the long-row searches (csrc/nns_many.hip) against the C
oracle, bit-exact (indices, row splits, distances):

* ops.radius_search / layers.RadiusSearch — per-query radii, rows in
  ascending (distance, index) order (oracle/o3d_oracle.c orc_radius_search);
  Open3D ml ops API (no reference model calls it), so parity
  with Open3D itself is unpinned;
* ops.knn_search with 64 < k <= 2048 batched over many queries (no host loop)
  and ignore_query_point for every k (the reference's knn_search API,
  point_transformer.py:724-729)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _cloud(n, seed=0, scale=1.0, offset=0.0):
    return (np.random.default_rng(seed).random((n, 3), dtype=np.float32) * scale + offset).astype(np.float32)


def _check(res, ref, with_dist=True):
    oi, ors, od = ref
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    if with_dist:
        assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


# ------------------------------------------------------------------ radius search
@pytest.mark.parametrize("metric", ["L2", "L1", "Linf"])
@pytest.mark.parametrize("ignore", [False, True])
def test_radius_search_batched(cuda, metric, ignore):
    from o3dml_amd import ops
    pts = _cloud(6000, 1, 2.0)
    pts[100:110] = pts[5]  # duplicates of a query position
    qry = np.concatenate([_cloud(900, 2, 2.4, -0.2), pts[:300]])
    radii = np.random.default_rng(3).uniform(0.02, 0.25, len(qry)).astype(np.float32)
    prs = np.array([0, 2500, 2500, 6000], np.int64)  # an empty batch item
    qrs = np.array([0, 500, 700, 1200], np.int64)
    res = ops.radius_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda),
                            torch.from_numpy(radii).to(cuda), torch.from_numpy(prs), torch.from_numpy(qrs),
                            metric=metric, ignore_query_point=ignore, return_distances=True)
    ref = O.radius_search(pts, qry, radii, prs, qrs, metric=metric, ignore_query_point=ignore,
                          return_distances=True)
    assert len(ref[0]) > 1000
    _check(res, ref)


def test_radius_search_normalized_int64_layer(cuda):
    from o3dml_amd import layers
    pts = _cloud(3000, 4)
    radii = np.full(3000, 0.08, np.float32)
    radii[::7] = 0.15
    t = torch.from_numpy(pts).to(cuda)
    res = layers.RadiusSearch(return_distances=True, normalize_distances=True, index_dtype=torch.int64)(
        t, t, torch.from_numpy(radii).to(cuda))
    ref = O.radius_search(pts, pts, radii, return_distances=True, normalize_distances=True, index_dtype=np.int64)
    assert res.neighbors_index.dtype == torch.int64
    _check(res, ref)


def test_radius_search_long_rows(cuda):
    """Rows longer than the 1,024- and 8,192-entry LDS lists (dense cluster):
    the large list and the unsorted-write + radix-sort path; no distances
    requested (the library then sorts through a scratch distance buffer)."""
    from o3dml_amd import ops
    pts = np.concatenate([_cloud(12000, 5, 0.05), _cloud(4000, 6, 1.0)])
    qry = np.concatenate([pts[:40], _cloud(60, 7)])
    radii = np.concatenate([np.full(20, 0.2), np.full(20, 0.02), np.full(60, 0.1)]).astype(np.float32)
    res = ops.radius_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda),
                            torch.from_numpy(radii).to(cuda))
    ref = O.radius_search(pts, qry, radii)
    rows = np.diff(ref[1])
    assert rows.max() > 8192 and ((rows > 1024) & (rows <= 8192)).any()
    assert res.neighbors_distance.numel() == 0
    _check(res, ref, with_dist=False)


def test_radius_search_empty(cuda):
    from o3dml_amd import ops
    pts = torch.from_numpy(_cloud(100, 8)).to(cuda)
    q = torch.zeros((0, 3), device=cuda)
    res = ops.radius_search(pts, q, torch.zeros(0, device=cuda))
    assert res.neighbors_index.numel() == 0 and res.neighbors_row_splits.tolist() == [0]
    res = ops.radius_search(torch.zeros((0, 3), device=cuda), pts, torch.full((100,), 0.1, device=cuda))
    assert res.neighbors_index.numel() == 0 and res.neighbors_row_splits.cpu().numpy().tolist() == [0] * 101


# ------------------------------------------------------------------ kNN k > 64
@pytest.mark.parametrize("k", [65, 200, 1024, 2048])
def test_knn_large_k_batched(cuda, k):
    """Thousands of queries with 64 < k <= 2048 in one batched launch."""
    from o3dml_amd import ops
    pts = _cloud(20000, k, 3.0)
    qry = np.concatenate([_cloud(1500, k + 1, 3.6, -0.3), pts[:500]])
    prs = np.array([0, 12000, 20000], np.int64)
    qrs = np.array([0, 1000, 2000], np.int64)
    res = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), k, torch.from_numpy(prs),
                         torch.from_numpy(qrs), return_distances=True)
    _check(res, O.knn_search(pts, qry, k, prs, qrs, return_distances=True))


def test_knn_large_k_surface_and_tiny_items(cuda):
    """Surface data (a 64-beam scan: candidate lists overflow on the dense
    ground near the sensor -> per-query path) and batch items with fewer
    points than k."""
    import bench
    from o3dml_amd import ops
    scan, _ = bench.make_scan(5)
    pts = np.concatenate([scan[:30000], _cloud(50, 9)])
    qry = np.concatenate([scan[:400], _cloud(20, 10)])
    prs = np.array([0, 30000, 30050], np.int64)
    qrs = np.array([0, 400, 420], np.int64)
    res = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), 1500, torch.from_numpy(prs),
                         torch.from_numpy(qrs), return_distances=True, index_dtype=torch.int64)
    _check(res, O.knn_search(pts, qry, 1500, prs, qrs, return_distances=True, index_dtype=np.int64))


@pytest.mark.parametrize("k", [100, 3000])
@pytest.mark.parametrize("metric", ["L2", "Linf"])
def test_knn_large_k_ignore_query_point(cuda, k, metric):
    """ignore_query_point for k > 64 (batched path at k = 100, per-query path
    at k = 3000), with duplicated query positions."""
    from o3dml_amd import ops
    pts = _cloud(8000, 12, 2.0)
    pts[50:60] = pts[3]
    qry = pts[:64].copy()
    res = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), k, metric=metric,
                         ignore_query_point=True, return_distances=True)
    _check(res, O.knn_search(pts, qry, k, metric=metric, ignore_query_point=True, return_distances=True))


# ------------------------------------------------------------------ radix selection (nns_topk.hip)
@pytest.mark.parametrize("mode", ["straddle", "whole_item"])
def test_knn_huge_k_ties_at_the_boundary(cuda, mode):
    """k > 2048 (radix selection + a sort of the k selected): 500 copies of
    one point make 500 keys equal; k is chosen so that the k-th neighbour
    falls inside that block (the selection must take the lowest indices among
    the ties), or exceeds batch item 0 (whole item); two queries in two
    batch items, int64 ids, distances."""
    from o3dml_amd import ops
    pts = _cloud(60000, 21, 4.0)
    pts[30000:30500] = pts[7]  # 500 copies of one point
    qry = np.stack([pts[7] + np.float32(0.9), pts[40000]])
    prs = np.array([0, 45000, 60000], np.int64)
    qrs = np.array([0, 1, 2], np.int64)
    oi, _, od = O.knn_search(pts[:45000], qry[:1], 45000, return_distances=True)
    first = int(np.flatnonzero(oi == 7)[0])
    k = first + 250 if mode == "straddle" else 45056
    assert k > 2048 and (mode != "straddle" or od[first + 250] == od[first])
    res = ops.knn_search(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), k, torch.from_numpy(prs),
                         torch.from_numpy(qrs), return_distances=True, index_dtype=torch.int64)
    _check(res, O.knn_search(pts, qry, k, prs, qrs, return_distances=True, index_dtype=np.int64))


def test_knn_select_set_index_order(cuda):
    """o3dml_knn_select (the captured RandLA crop): the k-nearest SET of the
    oracle's kNN in index order, with a block of duplicates at the k-th
    distance (lowest indices taken) and the whole cloud (k = n)."""
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr, stream_handle
    lib = _lib.load()
    pts = _cloud(70000, 23, 10.0)
    pts[100:400] = pts[5000]
    c = pts[5000] + np.float32(0.37)
    t = torch.from_numpy(pts).to(cuda)
    ct = torch.from_numpy(c).to(cuda)
    oi, _, od = O.knn_search(pts, c[None], 70000, return_distances=True)
    pos = np.flatnonzero(od == od[oi == 100][0])  # the duplicates' distance in the oracle's order
    for k in (int(pos[len(pos) // 2]) + 1, 45056, 70000):
        out = torch.empty(k, dtype=torch.int64, device=cuda)
        ws = torch.empty(lib.o3dml_knn_select_workspace_size(70000), dtype=torch.uint8, device=cuda)
        _lib.call("o3dml_knn_select", ptr(t), 70000, ptr(ct), k, 1, ptr(out), ptr(ws), ws.numel(), stream_handle(cuda))
        assert np.array_equal(out.cpu().numpy(), np.sort(oi[:k])), k


def test_knn_many_path_is_capturable(cuda):
    """64 < k <= 2048 count + fill (incl. the overflow queries' radix
    selection) inside a HIP graph capture, replayed several times with the
    queries changed between replays: no host synchronisation in the library,
    and every replay equals the oracle — the overflow counter and list are
    re-zeroed by a kernel on each replay (a hipMemsetAsync node of >= 16 bytes
    is re-applied on the first replay only on this runtime: csrc/fill.hip)."""
    import bench
    from o3dml_amd import _lib
    from o3dml_amd._util import ptr
    lib = _lib.load()
    scan, _ = bench.make_scan(5)
    pts = np.ascontiguousarray(scan[:30000])
    # dense ground: candidate lists overflow -> radix selection
    query_sets = [np.ascontiguousarray(scan[a:a + 400]) for a in (0, 1000, 0, 5000)]
    k = 1500
    prs = np.array([0, 30000], np.int64)
    qrs = np.array([0, 400], np.int64)
    pt, qt = torch.from_numpy(pts).to(cuda), torch.from_numpy(query_sets[0]).to(cuda)
    prs_d, qrs_d = torch.from_numpy(prs).to(cuda), torch.from_numpy(qrs).to(cuda)
    rs = torch.empty(401, dtype=torch.int64, device=cuda)
    idx = torch.empty(400 * k, dtype=torch.int32, device=cuda)
    dist = torch.empty(400 * k, dtype=torch.float32, device=cuda)
    ws = torch.empty(lib.o3dml_knn_search_workspace_size(30000, 400, k, 1), dtype=torch.uint8, device=cuda)
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        st = side.cuda_stream
        _lib.call("o3dml_knn_search_count", ptr(pt), 30000, ptr(qt), 400, k, 1, ptr(prs_d), ptr(qrs_d),
                  prs.ctypes.data, qrs.ctypes.data, 1, 0, 0, ptr(rs), ptr(ws), ws.numel(), st)
        _lib.call("o3dml_knn_search_fill", ptr(pt), 30000, ptr(qt), 400, k, 1, ptr(qrs_d), prs.ctypes.data,
                  qrs.ctypes.data, 1, 0, ptr(rs), 32, ptr(idx), ptr(dist), ptr(ws), ws.numel(), st)
    overflow = []
    for i, qry in enumerate(query_sets):
        qt.copy_(torch.from_numpy(qry))
        g.replay()
        torch.cuda.synchronize(cuda)
        overflow.append(int(ws[:8].view(torch.int64)[0]))
        oi, ors, od = O.knn_search(pts, qry, k, prs, qrs, return_distances=True)
        assert np.array_equal(rs.cpu().numpy(), ors), i
        assert np.array_equal(idx.cpu().numpy(), oi) and np.array_equal(dist.cpu().numpy(), od), i
    assert overflow[0] > 0  # some queries took the overflow path
    assert overflow[2] == overflow[0]  # the counter starts from zero on every replay


def test_knn_search_layer_point_transformer_shapes(cuda):
    """layers.KNNSearch as PointTransformer's knn_batch calls it
    (point_transformer.py:700-734: CPU tensors in, return_distances=True,
    reshape(-1, k)) at the model's shapes (:60 stride [1, 4, 4, 4, 4], nsample
    [8, 16, 16, 16, 16]) on two S3DIS-like clouds of 20,000 points: per level
    the self kNN of queryandgroup (k = nsample), the transition-down kNN
    (level l - 1 points, level l queries, k = 16) and the interpolation 3-NN
    (level l points, level l - 1 queries) — indices and distances bit-exact
    vs the oracle, results back on the CPU."""
    import bench
    from o3dml_amd import layers
    pts, _, _, lengths = bench.make_c3(0)
    rng = np.random.default_rng(9)
    levels = [(pts, np.array([0, lengths[0], lengths[0] + lengths[1]], np.int64))]
    for _ in range(4):  # stride 4: a subset of each item (FPS-sized)
        p, rs = levels[-1]
        keep, nrs = [], [0]
        for b in range(len(rs) - 1):
            nb = (rs[b + 1] - rs[b]) // 4
            keep.append(rs[b] + np.sort(rng.choice(rs[b + 1] - rs[b], nb, replace=False)))
            nrs.append(nrs[-1] + nb)
        levels.append((np.ascontiguousarray(p[np.concatenate(keep)]), np.array(nrs, np.int64)))
    nsample = [8, 16, 16, 16, 16]
    knn = layers.KNNSearch(return_distances=True)

    def check(points, prs, queries, qrs, k):
        ans = knn(torch.from_numpy(points), torch.from_numpy(queries), k, torch.from_numpy(prs),
                  torch.from_numpy(qrs))
        assert not ans.neighbors_index.is_cuda  # CPU in -> CPU out, as the caller expects
        oi, ors, od = O.knn_search(points, queries, k, prs, qrs, return_distances=True)
        assert np.array_equal(ans.neighbors_row_splits.numpy(), ors)
        assert np.array_equal(ans.neighbors_index.numpy(), oi), k
        assert np.array_equal(ans.neighbors_distance.numpy(), od), k
        assert ans.neighbors_index.reshape(-1, k).shape == (len(queries), k)

    for lvl, (p, rs) in enumerate(levels):
        check(p, rs, p, rs, nsample[lvl])
        if lvl > 0:
            fp, frs = levels[lvl - 1]
            check(fp, frs, p, rs, 16)  # transition down
            check(p, rs, fp, frs, 3)   # interpolation
