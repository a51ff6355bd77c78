"""GPU ops (HIP library via the C ABI) against the committed golden fixtures
(tests/golden/golden.npz): neighbour sets vs scipy, voxel ids vs numpy, and
the reference's own model plumbing (kpconv.batch_neighbors,
PointPillarsVoxelization, sparseconvnet InputLayer / calculate_grid)
re-run on this build's ops."""
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("tag", ["frs_uni", "frs_frag"])
def test_frs_vs_scipy_and_oracle(cuda, tag):
    from o3dml_amd import layers
    pts, r = G[f"{tag}_points"], float(G[f"{tag}_radius"])
    res = layers.FixedRadiusSearch(return_distances=True)(_t(pts, cuda), _t(pts, cuda), r)
    idx, rs = res.neighbors_index.cpu().numpy(), res.neighbors_row_splits.cpu().numpy()
    oi, ors, od = O.fixed_radius_search(pts, pts, r, return_distances=True)
    assert np.array_equal(rs, ors) and np.array_equal(idx, oi)
    assert np.array_equal(res.neighbors_distance.cpu().numpy(), od)
    sv, srs = G[f"{tag}_index"], G[f"{tag}_row_splits"]
    av, ars = G[f"{tag}_amb_index"], G[f"{tag}_amb_row_splits"]
    for q in range(len(pts)):
        diff = set(idx[rs[q]:rs[q + 1]].tolist()) ^ set(sv[srs[q]:srs[q + 1]].tolist())
        assert diff <= set(av[ars[q]:ars[q + 1]].tolist())


def test_knn_vs_scipy(cuda):
    from o3dml_amd import ops
    sup, qry = G["knn_sup"], G["knn_qry"]
    r = ops.knn_search(_t(sup, cuda), _t(qry, cuda), 16, return_distances=True)
    idx = r.neighbors_index.cpu().numpy().reshape(-1, 16)
    oi, _, _ = O.knn_search(sup, qry, 16, return_distances=True)
    assert np.array_equal(idx, oi.reshape(-1, 16))
    ref = G["knn_index"]
    bad = np.nonzero((idx != ref).any(1))[0]
    assert len(bad) <= 2
    np.testing.assert_allclose(r.neighbors_distance.cpu().numpy().reshape(-1, 16), G["knn_dist64"], rtol=1e-5,
                               atol=1e-7)


def test_voxelize_vs_numpy(cuda):
    from o3dml_amd import ops
    vp = G["vox_points"]
    res = ops.voxelize(_t(vp, cuda), torch.tensor([0, len(vp)]), G["vox_size"], G["vox_min"], G["vox_max"])
    c = res.voxel_coords.cpu().numpy().astype(np.int64)
    ext = ((G["vox_max"].astype(np.float64) - G["vox_min"].astype(np.float64)) *
           (1.0 / G["vox_size"].astype(np.float64))).astype(np.int32).astype(np.int64)
    assert np.array_equal(c[:, 0] + ext[0] * (c[:, 1] + ext[1] * c[:, 2]), G["vox_keys"])
    assert np.array_equal(np.diff(res.voxel_point_row_splits.cpu().numpy()), G["vox_counts"])


def test_grid_subsample_and_pointnet2(cuda):
    from o3dml_amd import contrib, ops
    assert np.array_equal(contrib.subsample(G["grid_points"], sampleDl=float(G["grid_dl"])), G["grid_expected"])
    fps = ops.furthest_point_sampling(_t(G["fps_points"], cuda), 64).cpu().numpy()
    assert np.array_equal(fps, G["fps_expected"])
    bq = ops.ball_query(_t(G["bq_xyz"], cuda), _t(G["bq_center"], cuda), 0.15, 8).cpu().numpy()
    assert np.array_equal(bq, G["bq_expected"])
    _, i = ops.three_nn(_t(G["bq_center"], cuda), _t(G["bq_xyz"], cuda))
    assert np.array_equal(i.cpu().numpy(), G["tnn_expected"])


def test_kpconv_batch_neighbors(cuda):
    """kpconv.py:2016-2034 on this build's ops (shadow index = N)."""
    from o3dml_amd import layers, ops
    pts, b, r = G["kpnb_points"], G["kpnb_batches"], float(G["kpnb_radius"])
    splits = torch.from_numpy(np.concatenate([[0], np.cumsum(b)]).astype(np.int64))
    p = _t(pts, cuda)
    res = layers.FixedRadiusSearch(return_distances=False)(p, p, r, splits, splits)
    rs = res.neighbors_row_splits
    dense = ops.ragged_to_dense(res.neighbors_index, rs, int((rs[1:] - rs[:-1]).max()),
                                torch.tensor(len(pts), dtype=torch.int32))
    assert np.array_equal(dense.cpu().numpy().astype(np.int64), G["kpnb_out"])


def test_pointpillars_voxelization(cuda):
    """point_pillars.py:352-382 on this build's ops."""
    from o3dml_amd import ops
    pf = _t(G["pillars_in"], cuda)
    res = ops.voxelize(pf[:, :3].contiguous(), torch.tensor([0, pf.shape[0]]), [0.16, 0.16, 4], [0, -39.68, -3],
                       [69.12, 39.68, 1], 32, 40000)
    dense = ops.ragged_to_dense(res.voxel_point_indices, res.voxel_point_row_splits, 32,
                                torch.tensor(-1, dtype=torch.int64)) + 1
    feats = torch.cat([torch.zeros_like(pf[:1]), pf])
    zyx = res.voxel_coords[:, [2, 1, 0]]
    keep = (zyx[:, 1] < 496) & (zyx[:, 2] < 432)
    num = res.voxel_point_row_splits[1:] - res.voxel_point_row_splits[:-1]
    assert np.array_equal(feats[dense][keep].cpu().numpy(), G["pillars_voxels"])
    assert np.array_equal(zyx[keep].cpu().numpy(), G["pillars_coords"])
    assert np.array_equal(num[keep].cpu().numpy(), G["pillars_num"])


def test_sparseconvnet_input_layer(cuda):
    """sparseconvnet.py:286-329 on this build's ops."""
    from o3dml_amd import ops
    pos, feat = _t(G["inputlayer_pos_in"], cuda), _t(G["inputlayer_feat_in"], cuda)
    res = ops.voxelize(pos, torch.tensor([0, pos.shape[0]]), [1, 1, 1], [0, 0, 0], [40960] * 3)
    pidx, prs = res.voxel_point_indices, res.voxel_point_row_splits
    assert np.array_equal(pos[pidx][prs[:-1]].cpu().numpy(), G["inputlayer_pos"])
    f = feat[pidx]
    cnt = (prs[1:] - prs[:-1]).float()
    avg = torch.stack([ops.reduce_subarrays_sum(f[:, c].contiguous(), prs) for c in range(3)], 1) / cnt[:, None]
    assert np.array_equal(avg.cpu().numpy(), G["inputlayer_feat"])


def test_calculate_grid(cuda):
    from o3dml_amd import ops
    assert np.array_equal(ops.calculate_grid(_t(G["calcgrid_in"], cuda)).cpu().numpy(), G["calcgrid_out"])
    rng = np.random.default_rng(5)
    # half-integer voxel centres plus arbitrary reals around zero (trunc edge)
    pos = np.concatenate([rng.integers(0, 3000, (200000, 3)) + 0.5,
                          rng.uniform(-3, 3, (5000, 3))]).astype(np.float32)
    assert np.array_equal(ops.calculate_grid(_t(pos, cuda)).cpu().numpy(), O.calculate_grid(pos))
    assert ops.calculate_grid(_t(np.zeros((0, 3), np.float32), cuda)).shape == (0, 3)
    with pytest.raises(RuntimeError):
        ops.calculate_grid(_t(np.full((4, 3), 3e6, np.float32), cuda))


@pytest.mark.parametrize("case", ["room", "flat", "wide", "negative", "one_cell"])
def test_calculate_grid_large_vs_oracle(cuda, case):
    """calculate_grid above the one-workgroup sort (n > 8,192: the multi-pass
    radix sort whose passes run only for the digits that vary among the packed
    parent keys, planned on the device) vs the oracle, bit-exact: the C4 room,
    a flat slab (one axis constant), coordinates over the whole 20-bit field
    range, points with negative coordinates (no parent) and every point in one
    parent cell (no digit varies)."""
    import bench
    from o3dml_amd import ops
    rng = np.random.default_rng(31)
    if case == "room":
        pos = bench.make_room(0)[0]
    elif case == "flat":
        pos = (np.stack([rng.integers(0, 300, 40000), rng.integers(0, 300, 40000), np.full(40000, 7)], 1)
               + 0.5).astype(np.float32)
    elif case == "wide":
        pos = (rng.integers(0, (1 << 21) - 2, (30000, 3)) + 0.5).astype(np.float32)
    elif case == "negative":
        pos = (rng.integers(-50, 50, (30000, 3)) + 0.5).astype(np.float32)
    else:
        pos = (np.full((20000, 3), 10) + rng.integers(0, 2, (20000, 3)) + 0.5).astype(np.float32)
    out = ops.calculate_grid(_t(pos, cuda)).cpu().numpy()
    assert np.array_equal(out, O.calculate_grid(pos))
