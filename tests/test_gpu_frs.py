"""GPU parity: fixed-radius search + spatial hash build vs the oracle
(bit-exact indices, row splits, hash tables; distances bit-exact too since both
sides use the same fmaf contraction)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _cloud(n, seed=0, scale=1.0):
    return (np.random.default_rng(seed).random((n, 3), dtype=np.float32) * scale).astype(np.float32)


def test_hash_table_bit_exact(cuda):
    from o3dml_amd import ops
    pts = _cloud(20000, 1)
    rs = np.array([0, 7000, 7000, 20000], np.int64)  # includes an empty batch item
    ht = ops.build_spatial_hash_table(torch.from_numpy(pts).to(cuda), 0.05, torch.from_numpy(rs))
    oi, oc, osp = O.build_spatial_hash_table(pts, 0.05, rs)
    assert np.array_equal(ht.hash_table_splits.numpy().astype(np.uint32), osp)
    assert np.array_equal(ht.hash_table_cell_splits.cpu().numpy().astype(np.uint32), oc)
    assert np.array_equal(ht.hash_table_index.cpu().numpy().astype(np.uint32), oi)


@pytest.mark.parametrize("metric", ["L2", "L1", "Linf"])
@pytest.mark.parametrize("ignore", [False, True])
def test_frs_self_search(cuda, metric, ignore):
    from o3dml_amd import layers
    pts = _cloud(16384, 0)
    pts[100] = pts[50]  # an exact duplicate exercises ignore_query_point
    nns = layers.FixedRadiusSearch(metric=metric, ignore_query_point=ignore, return_distances=True)
    t = torch.from_numpy(pts).to(cuda)
    res = nns(t, t, 0.06)
    oi, ors, od = O.fixed_radius_search(pts, pts, 0.06, metric=metric, ignore_query_point=ignore,
                                        return_distances=True)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


def test_frs_batched_queries_differ(cuda):
    from o3dml_amd import layers
    pts = _cloud(12000, 2, 2.0) - 0.5  # negative coordinates -> negative voxel ids
    qry = _cloud(5000, 3, 2.0) - 0.5
    prs = torch.LongTensor([0, 4000, 12000])
    qrs = torch.LongTensor([0, 3000, 5000])
    nns = layers.FixedRadiusSearch(index_dtype=torch.int64)
    res = nns(torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda), 0.1, prs, qrs)
    oi, ors, _ = O.fixed_radius_search(pts, qry, 0.1, prs.numpy(), qrs.numpy(), index_dtype=np.int64)
    assert res.neighbors_index.dtype == torch.int64
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)


def test_frs_c1_config(cuda):
    """BASELINE config 1: 65,536 U[0,1)^3 points (seed 0), r = 0.05."""
    from o3dml_amd import layers
    pts = np.random.default_rng(0).random((65536, 3), dtype=np.float32)
    t = torch.from_numpy(pts).to(cuda)
    res = layers.FixedRadiusSearch()(t, t, 0.05)
    oi, ors, _ = O.fixed_radius_search(pts, pts, 0.05)
    assert int(ors[-1]) == int(res.neighbors_row_splits[-1])
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)


def test_frs_cpu_tensors_roundtrip(cuda):
    """The reference calls the op with CPU tensors (kpconv.py:2021); results come back on CPU."""
    from o3dml_amd import layers
    pts = _cloud(3000, 5)
    res = layers.FixedRadiusSearch()(torch.from_numpy(pts), torch.from_numpy(pts), 0.08)
    assert not res.neighbors_index.is_cuda
    oi, ors, _ = O.fixed_radius_search(pts, pts, 0.08)
    assert np.array_equal(res.neighbors_index.numpy(), oi)


def test_frs_empty(cuda):
    from o3dml_amd import layers
    pts = torch.from_numpy(_cloud(100, 6)).to(cuda)
    empty = torch.zeros((0, 3), dtype=torch.float32, device=cuda)
    r1 = layers.FixedRadiusSearch()(pts, empty, 0.1)
    assert r1.neighbors_row_splits.cpu().tolist() == [0] and r1.neighbors_index.numel() == 0
    r2 = layers.FixedRadiusSearch()(empty, pts, 0.1)
    assert r2.neighbors_row_splits.cpu().numpy().tolist() == [0] * 101


def test_ragged_to_dense_and_reduce(cuda):
    from o3dml_amd import ops
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 9, 500)
    rs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    vals = rng.integers(0, 1000, rs[-1]).astype(np.int32)
    out = ops.ragged_to_dense(torch.from_numpy(vals.reshape(-1, 1)).to(cuda), torch.from_numpy(rs).to(cuda), 6,
                              torch.tensor([-7], dtype=torch.int32))
    ref = O.ragged_to_dense(vals.reshape(-1, 1), rs, 6, np.array([-7], np.int32))
    assert np.array_equal(out.cpu().numpy(), ref)
    v64 = torch.from_numpy(vals.astype(np.int64)).to(cuda)
    out2 = ops.ragged_to_dense(v64, torch.from_numpy(rs).to(cuda), 32, torch.tensor(-1)) + 1
    ref2 = O.ragged_to_dense(vals.astype(np.int64), rs, 32, np.int64(-1)) + 1
    assert np.array_equal(out2.cpu().numpy(), ref2)
    f = rng.standard_normal(rs[-1]).astype(np.float32)
    s = ops.reduce_subarrays_sum(torch.from_numpy(f).to(cuda), torch.from_numpy(rs).to(cuda))
    assert np.array_equal(s.cpu().numpy(), O.reduce_subarrays_sum(f, rs))


def test_frs_sparse_scene_hashed_grid(cuda):
    """Clusters far apart relative to r: the dense grid would be too large, the
    hashed fine grid path runs (and must still match the oracle bit for bit)."""
    from o3dml_amd import layers
    rng = np.random.default_rng(9)
    c = [rng.random((3000, 3), dtype=np.float32) * 0.5 + off for off in (0.0, 500.0, -800.0)]
    pts = np.concatenate(c).astype(np.float32)
    res = layers.FixedRadiusSearch(return_distances=True)(torch.from_numpy(pts).to(cuda),
                                                          torch.from_numpy(pts).to(cuda), 0.03)
    oi, ors, od = O.fixed_radius_search(pts, pts, 0.03, return_distances=True)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


def test_frs_extreme_coordinates_segment_path(cuda):
    """|coord| / r beyond the fine-grid range: the Open3D-cell segment path runs."""
    from o3dml_amd import layers
    rng = np.random.default_rng(10)
    pts = (rng.random((2000, 3)) * 1e-3 + 3e4).astype(np.float32)
    pts[1] = pts[0]
    res = layers.FixedRadiusSearch()(torch.from_numpy(pts).to(cuda), torch.from_numpy(pts).to(cuda), 1e-5)
    oi, ors, _ = O.fixed_radius_search(pts, pts, 1e-5)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)


def test_frs_dense_cluster_overflow_rows(cuda):
    """Rows longer than the 64-entry temp rows take the overflow re-run + long sort."""
    from o3dml_amd import layers
    rng = np.random.default_rng(11)
    pts = np.concatenate([rng.random((3000, 3), dtype=np.float32) * 0.02,
                          rng.random((5000, 3), dtype=np.float32)]).astype(np.float32)
    t = torch.from_numpy(pts).to(cuda)
    res = layers.FixedRadiusSearch(return_distances=True)(t, t, 0.05)
    oi, ors, od = O.fixed_radius_search(pts, pts, 0.05, return_distances=True)
    assert np.diff(ors).max() > 2000
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("sizes", [[65536, 1000], [70000, 3000], [1, 65536, 0, 40000]])
def test_frs_temp_row_widths(cuda, sizes):
    """Temp rows carry 16-bit ids relative to the batch item's first point when
    no item exceeds 65,536 points (the last id of a full item is 65,535) and
    32-bit ids otherwise; both must reproduce the oracle, with and without
    distances and for int64 output."""
    from o3dml_amd import layers
    rs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pts = np.concatenate([_cloud(max(n, 0), 10 + i) for i, n in enumerate(sizes)]) if rs[-1] else \
        np.zeros((0, 3), np.float32)
    t = torch.from_numpy(pts).to(cuda)
    for dist, dt in ((False, torch.int32), (True, torch.int64)):
        nns = layers.FixedRadiusSearch(return_distances=dist, index_dtype=dt)
        res = nns(t, t, 0.04, torch.from_numpy(rs), torch.from_numpy(rs))
        oi, ors, od = O.fixed_radius_search(pts, pts, 0.04, rs, rs, return_distances=dist,
                                            index_dtype=np.int64 if dt == torch.int64 else np.int32)
        assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
        assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
        if dist:
            assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("guess", [None, 0.0, 1e3])
def test_frs_speculative_capacity(cuda, guess):
    """The fill is queued into buffers sized from the last search's density
    before the host reads the total: no guess (read first), a guess far too
    small (bounded fill writes nothing, exact re-run) and far too large
    (sliced rows) all give the oracle's rows, plain and dense."""
    from o3dml_amd import ops
    pts = _cloud(20000, 31)
    pts[:300] = (0.5 + _cloud(300, 32) * 0.01).astype(np.float32)  # rows > 64: the overflow re-run (parts 2)
    rs = np.array([0, 12000, 20000], np.int64)
    t = torch.from_numpy(pts).to(cuda)
    r = 0.05
    for key in ((float(r), 1, len(pts), len(pts)), (float(r), -1, len(pts), len(pts))):
        ops._FRS_DENSITY.pop(key, None)
        if guess is not None:
            ops._FRS_DENSITY[key] = guess
    res = ops.fixed_radius_search(t, t, r, torch.from_numpy(rs), torch.from_numpy(rs), return_distances=True)
    oi, ors, od = O.fixed_radius_search(pts, pts, r, rs, rs, return_distances=True)
    assert res.neighbors_index.numel() == len(oi)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)
    dense = ops.fixed_radius_search_dense(t, t, r, torch.from_numpy(rs), torch.from_numpy(rs)).cpu().numpy()
    width = int(np.diff(ors).max())
    assert dense.shape == (len(pts), width)
    for q in (0, 777, 12000, 19999):
        row = oi[ors[q]:ors[q + 1]]
        assert np.array_equal(dense[q, :len(row)], row) and (dense[q, len(row):] == len(pts)).all()


@pytest.mark.parametrize("metric", ["L2", "L1", "Linf"])
def test_frs_group_sizes(cuda, metric):
    """Tight clusters of 1..64 points (each one query group of that size:
    floor(64 / size) lanes per query, sizes that are not powers of two
    included) among uniform points, with ignore_query_point and distances:
    rows equal the oracle's."""
    from o3dml_amd import ops
    rng = np.random.default_rng(7)
    parts = [_cloud(5000, 8)]
    for k in range(1, 65):
        c = rng.random(3, dtype=np.float32) * 0.9 + 0.05
        parts.append((c + rng.random((k, 3), dtype=np.float32) * 0.004).astype(np.float32))
    pts = np.concatenate(parts)
    rs = np.array([0, len(pts)], np.int64)
    t = torch.from_numpy(pts).to(cuda)
    for ignore in (False, True):
        res = ops.fixed_radius_search(t, t, 0.06, torch.from_numpy(rs), torch.from_numpy(rs), metric=metric,
                                      ignore_query_point=ignore, return_distances=True)
        oi, ors, od = O.fixed_radius_search(pts, pts, 0.06, rs, rs, metric=metric, ignore_query_point=ignore,
                                            return_distances=True)
        assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
        assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
        assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("factor,offset", [(1 / 512, 0.0), (1 / 64, 2700.0), (1 / 16, -3.0e5), (2.0, 0.0)])
def test_frs_voxel_classes(cuda, factor, offset):
    """The voxel-class sub-lists of the buckets: tables of 1/512 (many voxels
    per bucket: class 2 boxes), 1/16 and 2 bins per point (more bins than the
    class directory holds: whole buckets), coordinates ~2^17 voxels out
    (0.5-voxel box margins) and ~10^7 voxels out (no boxes): rows equal the
    oracle's on the same table, with distances, L2 and Linf."""
    from o3dml_amd import ops
    pts = (_cloud(30000, 51) + np.float32(offset)).astype(np.float32)
    rs = np.array([0, 12000, 30000], np.int64)
    r = 0.01
    t = torch.from_numpy(pts).to(cuda)
    ht = ops.build_spatial_hash_table(t, r, torch.from_numpy(rs), hash_table_size_factor=factor)
    oi_h, oc_h, osp_h = O.build_spatial_hash_table(pts, r, rs, hash_table_size_factor=factor)
    for metric in ("L2", "Linf"):
        res = ops.fixed_radius_search(t, t, r, torch.from_numpy(rs), torch.from_numpy(rs), ht.hash_table_splits,
                                      ht.hash_table_index, ht.hash_table_cell_splits, metric=metric,
                                      return_distances=True)
        ri, rr, rd = O.fixed_radius_search(pts, pts, r, rs, rs, hash_table=(oi_h, oc_h, osp_h), metric=metric,
                                           return_distances=True)
        assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), rr)
        assert np.array_equal(res.neighbors_index.cpu().numpy(), ri)
        assert np.array_equal(res.neighbors_distance.cpu().numpy(), rd)


@pytest.mark.parametrize("mode", ["1", "0"])
def test_frs_query_order(cuda, mode, monkeypatch):
    """Self search with the queries in Open3D's bucket order (the default for
    items below 2^22 points) and with the Morton-sorted queries of the general
    path (the default above), each forced on small items with empty and
    one-point items: the rows stay the oracle's."""
    from o3dml_amd import ops
    monkeypatch.setenv("O3DML_FRS_SELF_ORDER", mode)
    sizes = [30000, 0, 1, 45000]
    rs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pts = np.concatenate([_cloud(n, 40 + i) for i, n in enumerate(sizes) if n])
    t = torch.from_numpy(pts).to(cuda)
    res = ops.fixed_radius_search(t, t, 0.03, torch.from_numpy(rs), torch.from_numpy(rs), return_distances=True)
    oi, ors, od = O.fixed_radius_search(pts, pts, 0.03, rs, rs, return_distances=True)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


@pytest.mark.parametrize("n,rs_mid", [(300000, None), (90000, [5, 5, 40000]),
                                      (2200000, [5, 5] + [65536 * k for k in range(1, 33)])])
def test_hash_table_paths(cuda, n, rs_mid):
    """Both hash-table builders against the oracle: tables of > 4,096 bins in a
    batch item take the radix-sort path (300,000 points -> 4,687 bins), smaller
    ones the chunked counting sort — chunks of 1,024 points below 2^21 points
    per call (several chunks per item, empty and one-point items), of 4,096
    above (C1-shaped items) — each bit-exact; the FRS on top stays exact."""
    from o3dml_amd import ops
    pts = _cloud(n, 21)
    rs = np.array([0] + (rs_mid or []) + [n], np.int64)
    t = torch.from_numpy(pts).to(cuda)
    ht = ops.build_spatial_hash_table(t, 0.02, torch.from_numpy(rs))
    oi, oc, osp = O.build_spatial_hash_table(pts, 0.02, rs)
    assert np.array_equal(ht.hash_table_splits.numpy().astype(np.uint32), osp)
    assert np.array_equal(ht.hash_table_cell_splits.cpu().numpy().astype(np.uint32), oc)
    assert np.array_equal(ht.hash_table_index.cpu().numpy().astype(np.uint32), oi)
    if n > 1000000:
        return  # the oracle search would take minutes
    res = ops.fixed_radius_search(t, t, 0.02, torch.from_numpy(rs), torch.from_numpy(rs), ht.hash_table_splits,
                                  ht.hash_table_index, ht.hash_table_cell_splits)
    ri, rr, _ = O.fixed_radius_search(pts, pts, 0.02, rs, rs, hash_table=(oi, oc, osp))
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), rr)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), ri)


@pytest.mark.parametrize("guess", [None, 0.0, 1e3])
@pytest.mark.parametrize("dist,dt", [(False, torch.int32), (True, torch.int64)])
def test_frs_layer_one_call(cuda, guess, dist, dt):
    """layers.FixedRadiusSearch without a given table runs the table build,
    count, totals and speculative row copy as one library call
    (o3dml_fixed_radius_search_layer): no capacity guess, a guess far too small
    (exact re-run) and far too large (sliced rows), with rows longer than 64
    (the overflow re-run), an empty item, different queries and a repeated
    layout (cached plan) — every result equals the oracle's."""
    from o3dml_amd import layers, ops
    pts = _cloud(20000, 61)
    pts[:300] = (0.5 + _cloud(300, 62) * 0.01).astype(np.float32)
    qry = _cloud(7000, 63)
    rs = np.array([0, 12000, 12000, 20000], np.int64)
    qs = np.array([0, 3000, 3000, 7000], np.int64)
    r = 0.05
    t, tq = torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda)
    nns = layers.FixedRadiusSearch(return_distances=dist, index_dtype=dt)
    idt = np.int64 if dt == torch.int64 else np.int32
    for a, b, ars, brs in ((t, t, rs, rs), (t, tq, rs, qs), (t, t, rs, rs)):
        key = (float(r), 1, a.shape[0], b.shape[0])
        ops._FRS_DENSITY.pop(key, None)
        if guess is not None:
            ops._FRS_DENSITY[key] = guess
        res = nns(a, b, r, torch.from_numpy(ars), torch.from_numpy(brs))
        oi, ors, od = O.fixed_radius_search(a.cpu().numpy(), b.cpu().numpy(), r, ars, brs, return_distances=dist,
                                            index_dtype=idt)
        assert res.neighbors_index.dtype == dt and res.neighbors_index.numel() == len(oi)
        assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
        assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)
        if dist:
            assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)


def test_frs_dense_one_call(cuda):
    """KPConv's batch_neighbors through the one-call path: the dense matrix
    written straight from the temp rows (rows longer than 64 by the re-run at
    row * width), a table shared with a second search over the same supports,
    and an empty query set — equal to the oracle rows padded with the shadow
    index."""
    from o3dml_amd import kpfcnn
    pts = _cloud(9000, 71)
    pts[:200] = (0.3 + _cloud(200, 72) * 0.01).astype(np.float32)  # rows > 64
    qry = _cloud(3000, 73)
    sl, ql = [5000, 4000], [1000, 2000]
    t, tq = torch.from_numpy(pts).to(cuda), torch.from_numpy(qry).to(cuda)
    rs = np.array([0, 5000, 9000], np.int64)
    qs = np.array([0, 1000, 3000], np.int64)
    reads = kpfcnn._Reads(cuda)
    a = kpfcnn._dense_begin(reads, t, t, sl, sl, 0.05)
    b = kpfcnn._dense_begin(reads, tq, t, ql, sl, 0.05, a)
    e = kpfcnn._dense_begin(reads, tq[:0], t, [0, 0], sl, 0.05, a)
    host = reads.read()
    for x, h, q, qrs in ((a, host[0:3], pts, rs), (b, host[3:6], qry, qs)):
        d = kpfcnn._dense_end(x, h).cpu().numpy()
        oi, ors, _ = O.fixed_radius_search(pts, q, 0.05, rs, qrs)
        w = int(np.diff(ors).max())
        assert h[2] == w and d.shape == (len(q), w)
        assert h[0] == len(oi) and (h[1] > 0) == (w > 64)
        for i in range(len(q)):
            row = oi[ors[i]:ors[i + 1]]
            assert np.array_equal(d[i, :len(row)], row) and (d[i, len(row):] == len(pts)).all()
    assert kpfcnn._dense_end(e, host[6:9]).shape[0] == 0


def test_frs_bench_batch_bit_exact(cuda):
    """The exact batch bench.py times (64 scenes x 65,536 points, one call,
    u16 temp rows across 64 batch items) through layers.FixedRadiusSearch,
    twice (the second call takes the speculative capacity of the first), vs
    the oracle's fixed_radius_search on the same batch: bit-exact."""
    import bench
    from o3dml_amd import layers
    pts, rs = bench.make_batch(0, 64, cuda)
    nns = layers.FixedRadiusSearch()
    for _ in range(2):
        res = nns(pts, pts, bench.RADIUS, rs, rs)
    p = pts.cpu().numpy()
    oi, ors, _ = O.fixed_radius_search(p, p, bench.RADIUS, rs.numpy(), rs.numpy())
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)


@pytest.mark.parametrize("lg", [18, 20, 22])
def test_frs_large_item_bit_exact(cuda, lg):
    """One batch item of more than 65,536 points (the c1_sweep shapes of
    bench.py: N = 2^lg at the C1 density) vs the oracle, bit-exact."""
    from o3dml_amd import layers
    n = 1 << lg
    pts = np.random.default_rng(lg).random((n, 3), dtype=np.float32)
    r = 0.05 * (65536.0 / n) ** (1.0 / 3.0)
    t = torch.from_numpy(pts).to(cuda)
    res = layers.FixedRadiusSearch()(t, t, r)
    oi, ors, _ = O.fixed_radius_search(pts, pts, r)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert np.array_equal(res.neighbors_index.cpu().numpy(), oi)


def test_frs_2_24_sweep_scene_bit_exact(cuda):
    """The 2^24-point c1_sweep scene (bench.py c1_sweep: U[0,1)^3, seed 24,
    r = 0.05 (65536 / N)^(1/3); u32 temp rows, Morton query order) through
    layers.FixedRadiusSearch, twice as the sweep calls it, vs the optimised
    CPU search of the same semantics (oracle/cpu_frs.c, bit-identical to the
    oracle: tests/test_golden.py::test_cpu_frs_fast_equals_oracle): row splits
    and every neighbour index bit-exact (~560 M pairs, compared on the GPU)."""
    from o3dml_amd import layers
    n = 1 << 24
    pts = np.random.default_rng(24).random((n, 3), dtype=np.float32)
    r = 0.05 * (65536.0 / n) ** (1.0 / 3.0)
    t = torch.from_numpy(pts).to(cuda)
    rs = torch.tensor([0, n], dtype=torch.int64)
    nns = layers.FixedRadiusSearch()
    for _ in range(2):
        res = nns(t, t, r, rs, rs)
    oi, ors = O.fixed_radius_search_fast(pts, r, rs.numpy())
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert res.neighbors_index.shape[0] == len(oi)
    assert torch.equal(res.neighbors_index, torch.from_numpy(oi).to(cuda))


def test_frs_two_large_items_bit_exact(cuda):
    """Two batch items of ~2^22 points in one call (the Morton query order of
    large self searches keys the bucket-order points with batch bits), vs
    the optimised CPU search (= the oracle), bit-exact."""
    from o3dml_amd import layers
    sizes = [(1 << 22) + 3, (1 << 22) - 5]
    rng = np.random.default_rng(23)
    pts = np.concatenate([rng.random((n, 3), dtype=np.float32) + np.float32(i * 0.25) for i, n in enumerate(sizes)])
    rs = np.array([0, sizes[0], sizes[0] + sizes[1]], np.int64)
    r = 0.05 * (65536.0 / sizes[0]) ** (1.0 / 3.0)
    t = torch.from_numpy(pts).to(cuda)
    res = layers.FixedRadiusSearch()(t, t, r, torch.from_numpy(rs), torch.from_numpy(rs))
    oi, ors = O.fixed_radius_search_fast(pts, r, rs)
    assert np.array_equal(res.neighbors_row_splits.cpu().numpy(), ors)
    assert torch.equal(res.neighbors_index, torch.from_numpy(oi).to(cuda))
