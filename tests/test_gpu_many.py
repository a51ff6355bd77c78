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
