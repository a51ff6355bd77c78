"""Generate tests/golden/golden.npz (run in the build container only).

Two kinds of fixtures pin the CPU oracle (oracle/o3d_oracle.c):

A. Independent exact oracles — same inputs, answers from other code:
   scipy cKDTree in float64 (fixed-radius sets, kNN), numpy float64 voxel
   maths, numpy float32 restatement of KPConv grid subsampling, numpy greedy
   FPS / ball query / three-NN.  Inputs include a crop of the reference's own
   demo scan (data/demo/fragment.pcd, a real indoor scan).
B. Reference plumbing — the reference's own Python (ml3d, imported here via
   tools/ref_loader.py with the absent Open3D ops backed by the oracle):
   sparseconvnet.calculate_grid, PointPillarsVoxelization.forward,
   kpconv.batch_neighbors, sparseconvnet.InputLayer.forward.  These pin the
   argument meaning and output layout the models expect around the ops.

Only data (inputs and expected outputs) is written; no reference source.
"""
import os
import sys

import numpy as np
import torch
from scipy.spatial import cKDTree

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def csr(lists):
    rs = np.zeros(len(lists) + 1, np.int64)
    rs[1:] = np.cumsum([len(x) for x in lists])
    vals = np.concatenate([np.asarray(x, np.int64) for x in lists]) if rs[-1] else np.zeros(0, np.int64)
    return vals, rs


def load_fragment():
    path = "/root/reference/data/demo/fragment.pcd"
    raw = open(path, "rb").read()
    head, _, body = raw.partition(b"DATA binary\n")
    n = int([ln for ln in head.decode().splitlines() if ln.startswith("POINTS")][0].split()[1])
    arr = np.frombuffer(body[: n * 32], np.float32).reshape(n, 8)
    return np.ascontiguousarray(arr[:, :3])


def frs_fixture(out, tag, pts, r):
    t = cKDTree(pts.astype(np.float64))
    lists = [sorted(x) for x in t.query_ball_point(pts.astype(np.float64), r)]
    vals, rs = csr(lists)
    # pairs whose float64 distance is within 1e-5 relative of r are "boundary":
    # fp32 and fp64 may legitimately disagree on them
    t2 = t.query_ball_point(pts.astype(np.float64), r * (1 + 1e-5))
    t3 = t.query_ball_point(pts.astype(np.float64), r * (1 - 1e-5))
    amb = [sorted(set(a) - set(b)) for a, b in zip(t2, t3)]
    av, ars = csr(amb)
    out[f"{tag}_points"] = pts.astype(np.float32)
    out[f"{tag}_radius"] = np.float32(r)
    out[f"{tag}_index"], out[f"{tag}_row_splits"] = vals, rs
    out[f"{tag}_amb_index"], out[f"{tag}_amb_row_splits"] = av, ars


def grid_subsample_f32(points, dl):
    """numpy float32 restatement of KPConv grid_subsampling (barycentres),
    output in ascending cell-key order."""
    p = points.astype(np.float32)
    dl = np.float32(dl)
    inv = np.float32(1) / dl
    mn, mx = p.min(0), p.max(0)
    org = (np.floor(mn * inv) * dl).astype(np.float32)
    nx = np.uint64(np.floor((mx[0] - org[0]) / dl)) + np.uint64(1)
    ny = np.uint64(np.floor((mx[1] - org[1]) / dl)) + np.uint64(1)
    ijk = np.floor((p - org) / dl).astype(np.uint64)
    keys = ijk[:, 0] + nx * ijk[:, 1] + nx * ny * ijk[:, 2]
    order = np.argsort(keys, kind="stable")
    uniq = np.unique(keys)
    res = np.zeros((len(uniq), 3), np.float32)
    pos = {k: i for i, k in enumerate(uniq.tolist())}
    sums = np.zeros((len(uniq), 3), np.float32)
    cnt = np.zeros(len(uniq), np.int64)
    for i in order:  # input order within a cell (stable)
        c = pos[int(keys[i])]
        sums[c] = (sums[c] + p[i]).astype(np.float32)
        cnt[c] += 1
    for c in range(len(uniq)):
        res[c] = sums[c] * np.float32(1.0 / cnt[c])
    return res


def main():
    out = {}
    rng = np.random.default_rng(20251015)
    # ---------------- A: independent oracles
    frs_fixture(out, "frs_uni", rng.random((2048, 3), dtype=np.float32), 0.1)
    frag = load_fragment()
    box = (frag[:, 0] > np.percentile(frag[:, 0], 40)) & (frag[:, 0] < np.percentile(frag[:, 0], 46))
    crop = frag[box][:4000]
    frs_fixture(out, "frs_frag", crop, 0.1)
    sup = rng.random((3000, 3), dtype=np.float32)
    qry = rng.random((1500, 3), dtype=np.float32)
    d, i = cKDTree(sup.astype(np.float64)).query(qry.astype(np.float64), 16)
    out.update(knn_sup=sup, knn_qry=qry, knn_index=i.astype(np.int64), knn_dist64=d ** 2)
    vp = np.stack([rng.uniform(-1, 70, 4000), rng.uniform(-40, 40, 4000), rng.uniform(-3.2, 1.2, 4000)],
                  1).astype(np.float32)
    vs, vmn, vmx = np.array([0.16, 0.16, 4.0], np.float32), np.array([0, -39.68, -3], np.float32), \
        np.array([69.12, 39.68, 1], np.float32)
    inv = 1.0 / vs.astype(np.float64)
    ext = ((vmx.astype(np.float64) - vmn) * inv).astype(np.int32).astype(np.int64)
    c = np.floor((vp.astype(np.float64) - vmn.astype(np.float64)) * inv)
    ok = np.all((c >= 0) & (c < ext), 1)
    key = (c[:, 0] + ext[0] * (c[:, 1] + ext[1] * c[:, 2])).astype(np.int64)
    uk, cnt = np.unique(key[ok], return_counts=True)
    out.update(vox_points=vp, vox_size=vs, vox_min=vmn, vox_max=vmx, vox_keys=uk, vox_counts=cnt.astype(np.int64))
    gp = (rng.random((3000, 3)) * [3, 3, 1] - [1.5, 1.5, 0.2]).astype(np.float32)
    out.update(grid_points=gp, grid_dl=np.float32(0.06), grid_expected=grid_subsample_f32(gp, 0.06))
    fx = rng.random((1, 1500, 3)).astype(np.float32)
    x = fx[0].astype(np.float64)
    md = np.full(len(x), 1e10)
    sel = [0]
    for _ in range(63):
        md = np.minimum(md, ((x - x[sel[-1]]) ** 2).sum(1))
        sel.append(int(np.argmax(md)))
    out.update(fps_points=fx, fps_expected=np.asarray([sel], np.int32))
    bx = rng.random((1, 800, 3)).astype(np.float32)
    bc = rng.random((1, 100, 3)).astype(np.float32)
    d2 = ((bc[0, :, None, :].astype(np.float64) - bx[0, None, :, :]) ** 2).sum(-1)
    bq = np.zeros((1, 100, 8), np.int32)
    for j in range(100):
        hits = np.nonzero(d2[j] < 0.15 ** 2)[0][:8]
        if len(hits):
            bq[0, j, :] = hits[0]
            bq[0, j, :len(hits)] = hits
    tn = np.argsort(d2, 1, kind="stable")[:, :3]
    out.update(bq_xyz=bx, bq_center=bc, bq_expected=bq, tnn_expected=tn[None].astype(np.int32))
    # ---------------- B: reference plumbing (ref_loader)
    import ref_loader
    ref_loader.install()
    from ml3d.torch.models import kpconv, point_pillars, sparseconvnet
    vox = np.unique(rng.integers(0, 20, (2500, 3)), axis=0).astype(np.float32) + 0.5
    out["calcgrid_in"] = vox
    out["calcgrid_out"] = sparseconvnet.calculate_grid(torch.from_numpy(vox)).numpy()
    layer = point_pillars.PointPillarsVoxelization(voxel_size=[0.16, 0.16, 4],
                                                   point_cloud_range=[0, -39.68, -3, 69.12, 39.68, 1],
                                                   max_num_points=32, max_voxels=[16000, 40000]).eval()
    pf = np.concatenate([vp, rng.random((4000, 1), dtype=np.float32)], 1)
    ov, oc, on = layer(torch.from_numpy(pf))
    out.update(pillars_in=pf, pillars_voxels=ov.numpy(), pillars_coords=oc.numpy(), pillars_num=on.numpy())
    sub_a = crop[:2500]
    q_b, s_b = np.array([1200, 1300], np.int32), np.array([1200, 1300], np.int32)
    nb = kpconv.batch_neighbors(sub_a, sub_a, q_b, s_b, 0.1)
    out.update(kpnb_points=sub_a, kpnb_batches=q_b, kpnb_radius=np.float32(0.1), kpnb_out=nb.astype(np.int64))
    ip = (rng.random((3000, 3)) * 30).astype(np.float32)
    ifeat = rng.random((3000, 3)).astype(np.float32)
    fa, pos, imap = sparseconvnet.InputLayer()(torch.from_numpy(ifeat), torch.from_numpy(ip))
    out.update(inputlayer_pos_in=ip, inputlayer_feat_in=ifeat, inputlayer_feat=fa.numpy(),
               inputlayer_pos=pos.numpy(), inputlayer_map=np.asarray(imap, np.int64))
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
