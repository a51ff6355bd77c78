"""Generate tests/golden/full.npz (build container only): reference outputs at
the FULL sizes the bench times, data only.

C2 (SemanticKITTI-shaped scan, bench.make_scan(0), 120,000 points):
  * the sub-cloud = the oracle's contrib.subsample (grid 0.06, the reference's
    randlanet.py:133-139) — stored as a sha256 the GPU grid subsampling must
    reproduce, plus its size;
  * sklearn KDTree (float64, as randlanet.py:141 / semseg_spatially_regular.py
    :94-95 use it): the k = 45,056 patch crops around three centres and the
    1-NN projection of every raw point (randlanet.py:148-152).  Near-ties are
    tagged: crop entries whose float64 squared distance is within 1e-6
    (relative) of the crop's last one, projection queries whose two nearest
    squared distances are within 1e-6 — float32 and float64 may order those
    differently;
  * the reference RandLANet (randlanet.py, tools/ref_loader.py) on one full
    45,056-point patch (the oracle crop of centre 0 — bit-exact with the GPU
    kNN — in a seeded permutation, recentred as the augmenter does), per-layer
    neighbours from the oracle kNN (checked here against scipy float64 sets),
    deterministic weights (randla_weights.fill): every 11th row of the logits
    and the float64 column sums of all of them.
C3 (bench.make_c3(0), 40,000 points, KPFCNN kpconv_s3dis.yml at
  first_features_dim 128): the reference collate (concat_batcher.py:186-283,
  seeded np.random rotations recorded) as per-array sha256 + shapes, the
  kernel-point dispositions, and in eval and training mode: every 10th logit
  row, the logit column sums, the cross-entropy loss, the float64 L2 norm of
  every parameter gradient and the full gradient of the smallest tensors —
  of the reference in float32 AND of the same reference model run in float64
  (the truth), with the reference's own float32 error against it.
C4 (bench.make_room(0), 88,006 voxels, SparseConvUnet m=32 residual, 20
  classes, eval): every 11th logit row and the column sums."""
import hashlib
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402

C2_K = 45056
C2_CENTERS = (1000, 40000, 77777)  # sub-cloud indices of the crop centres
C2_PERM_SEED = 5
TIE_REL = 1e-6
C3_CFG = dict(lbl_values=list(range(13)), num_classes=13, ignored_label_inds=[], first_subsampling_dl=0.04,
              in_features_dim=5, first_features_dim=128, batch_norm_momentum=0.98, conv_radius=2.5,
              KP_extent=1.2, num_kernel_points=15)
C3_FULL_GRADS = ("head_softmax.mlp.weight", "head_mlp.mlp.weight", "encoder_blocks.0.KPConv.weights")
C4_FEAT_SEED = 3


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def c2_patch(sub):
    """The full-size patch of the forward check (also rebuilt by the test)."""
    import oracle as O
    c = C2_CENTERS[0]
    crop, _, _ = O.knn_search(sub, sub[c:c + 1], C2_K)
    perm = np.random.default_rng(C2_PERM_SEED).permutation(C2_K)
    pc = sub[crop.astype(np.int64)][perm].copy()
    pc[:, :2] -= pc[:, :2].mean(0, dtype=np.float64).astype(np.float32)
    return pc.astype(np.float32)


def c2_levels(pc):
    """Per-layer inputs of RandLANet (randlanet.py:212-239): kNN k=16 on each
    level, level i+1 = the first N_i/4 points, 1-NN up-sampling indices; the
    oracle kNN (bit-exact with the GPU's)."""
    import oracle as O
    coords, nbrs, subs, ups = [], [], [], []
    cur = pc
    for _ in range(4):
        nb, _, _ = O.knn_search(cur, cur, 16)
        nb = nb.reshape(-1, 16).astype(np.int64)
        sub = cur[: cur.shape[0] // 4]
        up, _, _ = O.knn_search(sub, cur, 1)
        coords.append(cur)
        nbrs.append(nb)
        subs.append(nb[: cur.shape[0] // 4])
        ups.append(up.reshape(-1, 1).astype(np.int64))
        cur = sub
    return coords, nbrs, subs, ups


def check_sets_vs_scipy(pts, nb, k):
    """Oracle kNN sets vs scipy float64 sets: every differing row must be a
    float64 tie at the k-th boundary."""
    from scipy.spatial import cKDTree
    d, i = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k + 1)
    bad = 0
    for r in np.flatnonzero(np.any(np.sort(nb, 1) != np.sort(i[:, :k], 1), 1)):
        if not (d[r, k] ** 2 - d[r, k - 1] ** 2 <= TIE_REL * d[r, k] ** 2):
            bad += 1
    return bad


def make_c2(out):
    import bench
    import oracle as O
    from sklearn.neighbors import KDTree
    scan, _ = bench.make_scan(0)
    sub = O.subsample(scan, sampleDl=0.06).astype(np.float32)
    out["c2_sub_sha"] = np.array(sha(sub))
    out["c2_sub_n"] = np.int64(len(sub))
    tree = KDTree(sub)
    s64 = sub.astype(np.float64)
    for j, c in enumerate(C2_CENTERS):
        idx = tree.query(sub[c:c + 1], k=C2_K)[1][0]
        d = ((s64 - s64[c]) ** 2).sum(1)
        kth = d[idx[-1]]
        out[f"c2_crop{j}"] = idx.astype(np.int32)
        out[f"c2_crop{j}_amb"] = np.flatnonzero(np.abs(d - kth) <= TIE_REL * kth).astype(np.int32)
    dd, ii = tree.query(scan, k=2)
    out["c2_proj"] = ii[:, 0].astype(np.int32)
    out["c2_proj_amb"] = np.flatnonzero(dd[:, 1] ** 2 - dd[:, 0] ** 2 <= TIE_REL * dd[:, 1] ** 2).astype(np.int32)
    print("c2 sub", len(sub), "crop amb", [len(out[f"c2_crop{j}_amb"]) for j in range(3)],
          "proj amb", len(out["c2_proj_amb"]))

    from ml3d.torch.models.randlanet import RandLANet
    pc = c2_patch(sub)
    coords, nbrs, subs, ups = c2_levels(pc)
    for i in range(4):
        bad = check_sets_vs_scipy(coords[i], nbrs[i], 16)
        assert bad == 0, (i, bad)
    torch.manual_seed(0)
    model = RandLANet(num_points=C2_K, num_classes=19, in_channels=3)
    sd = model.state_dict()
    model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()]))
    model.eval()
    model.device = torch.device("cpu")
    t = lambda a: torch.from_numpy(a)[None]  # noqa: E731
    inputs = {"coords": [t(c) for c in coords], "neighbor_indices": [t(n) for n in nbrs],
              "sub_idx": [t(s) for s in subs], "interp_idx": [t(u) for u in ups], "features": t(pc)}
    with torch.no_grad():
        logits = model(inputs)[0].numpy().astype(np.float32)
    out["c2_logit_rows"] = logits[::11]
    out["c2_logit_colsum"] = logits.astype(np.float64).sum(0)
    print("c2 logits", logits.shape, float(np.abs(logits).mean()))
    # the same reference model in float64 (same neighbours, same weights): the
    # truth the per-element C2 check holds fp32 results to, and the
    # reference's own fp32 error against it (as C3 / C4)
    model64 = RandLANet(num_points=C2_K, num_classes=19, in_channels=3)  # (its Config defeats deepcopy)
    model64.load_state_dict(model.state_dict())
    model64 = model64.double().eval()
    model64.device = torch.device("cpu")
    t64 = lambda a: torch.from_numpy(a)[None].double()  # noqa: E731
    inputs64 = dict(inputs, coords=[t64(c) for c in coords], features=t64(pc))
    with torch.no_grad():
        logits64 = model64(inputs64)[0].numpy()
    out["c2_f64_logit_rows"] = logits64[::11]
    out["c2_f64_logit_colsum"] = logits64.sum(0)
    err = np.abs(logits.astype(np.float64) - logits64)
    out["c2_ref32_abs_err"] = np.float64(err.max())
    out["c2_ref32_rel_err"] = np.float64((err / np.maximum(np.abs(logits64), 1e-300)).max())
    # per-row scale of the logits (max |logit| of the row): the floor of the
    # per-element check is a multiple of the reference's own fp32 error
    # relative to it
    out["c2_ref32_err_vs_rowmax"] = np.float64((err / np.abs(logits64).max(1, keepdims=True)).max())
    print("c2 ref fp32 vs fp64: max abs", float(out["c2_ref32_abs_err"]), "max rel", float(out["c2_ref32_rel_err"]),
          "vs row max", float(out["c2_ref32_err_vs_rowmax"]), "max |f64|", float(np.abs(logits64).max()))


def make_c3(out):
    import bench
    os.chdir("/tmp")  # load_kernels writes its kernel dispositions relative to the cwd
    import ml3d.torch.models.kpconv as K
    from ml3d.torch.dataloaders.concat_batcher import KPConvBatch
    pts, feats, labels, lengths = bench.make_c3(0)
    model = K.KPFCNN(**C3_CFG)
    cfg = model.cfg
    rots = []
    orig = K.create_3D_rotations

    def rec(axis, angle):
        R = orig(axis, angle)
        rots.append(R.astype(np.float32))
        return R
    K.create_3D_rotations = rec
    np.random.seed(0)
    fake = types.SimpleNamespace(cfg=cfg, neighborhood_limits=[])
    fake.big_neighborhood_filter = lambda nb, layer: nb
    t0 = time.time()
    li = KPConvBatch.segmentation_inputs(fake, pts, feats, labels, lengths)
    print("c3 collate", round(time.time() - t0, 1), "s")
    K.create_3D_rotations = orig
    L = cfg.num_layers
    out["c3_rotations"] = np.stack(rots)
    names = ["layer_points", "neighbors", "pools", "upsamples", "layer_lengths"]
    for gi, name in enumerate(names):
        for l in range(L):
            a = np.asarray(li[gi * L + l]).astype(np.float32 if name == "layer_points" else np.int32)
            out[f"c3_sha_{name}_{l}"] = np.array(sha(a))
            out[f"c3_shape_{name}_{l}"] = np.array(a.shape, np.int64)
    batch = types.SimpleNamespace(
        points=[torch.from_numpy(li[l]) for l in range(L)],
        neighbors=[torch.from_numpy(li[L + l]) for l in range(L)],
        pools=[torch.from_numpy(li[2 * L + l]) for l in range(L)],
        upsamples=[torch.from_numpy(li[3 * L + l]) for l in range(L)],
        lengths=[torch.from_numpy(li[4 * L + l]) for l in range(L)],
        features=torch.from_numpy(feats), labels=torch.from_numpy(labels))
    sd = model.state_dict()
    new = randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd)
    for k in sd:
        if k.endswith("kernel_points"):
            new[k] = sd[k].clone()
            out["c3_kp:" + k] = sd[k].numpy().astype(np.float32)
    model.load_state_dict(new)
    import copy
    model64 = copy.deepcopy(model).double()
    batch64 = types.SimpleNamespace(**{**batch.__dict__, "points": [p.double() for p in batch.points],
                                       "features": batch.features.double()})
    for mode in ("eval", "train"):
        res = {}
        for tag, mdl, b in (("", model, batch), ("64", model64, batch64)):
            mdl.zero_grad()
            mdl.train(mode == "train")
            t0 = time.time()
            logits = mdl(b)
            loss = torch.nn.functional.cross_entropy(logits, b.labels)
            loss.backward()
            print("c3", mode, tag or "32", round(time.time() - t0, 1), "s, loss", float(loss))
            lg = logits.detach().double().numpy()
            res[tag] = {"rows": lg[::10], "colsum": lg.sum(0), "loss": float(loss.item()),
                        "names": [], "norms": [], "full": {}}
            for k, p in mdl.named_parameters():
                if p.grad is None:
                    continue
                res[tag]["names"].append(k)
                res[tag]["norms"].append(float(np.linalg.norm(p.grad.double().numpy())))
                if k in C3_FULL_GRADS:
                    res[tag]["full"][k] = p.grad.double().numpy()
        r32, r64 = res[""], res["64"]
        assert r32["names"] == r64["names"]
        out[f"c3_{mode}_logit_rows"] = r32["rows"].astype(np.float32)
        out[f"c3_{mode}_logit_colsum"] = r32["colsum"]
        out[f"c3_{mode}_loss"] = np.float64(r32["loss"])
        out[f"c3_{mode}_grad_names"] = np.array(r32["names"])
        out[f"c3_{mode}_grad_norms"] = np.array(r32["norms"], np.float64)
        for k, g in r32["full"].items():
            out[f"c3_{mode}_grad:{k}"] = g.astype(np.float32)
        # the float64 run of the same reference model: the truth the fp32
        # results are held to, and the reference's own fp32 error against it
        out[f"c3_{mode}_f64_logit_rows"] = r64["rows"]
        out[f"c3_{mode}_f64_loss"] = np.float64(r64["loss"])
        out[f"c3_{mode}_f64_grad_norms"] = np.array(r64["norms"], np.float64)
        for k, g in r64["full"].items():
            out[f"c3_{mode}_f64_grad:{k}"] = g
        rel = lambda a, b: float(np.abs(a - b).max() / (np.abs(b).max() + 1e-300))  # noqa: E731
        out[f"c3_{mode}_ref32_err_rows"] = np.float64(rel(r32["rows"], r64["rows"]))
        out[f"c3_{mode}_ref32_err_norms"] = np.abs(np.array(r32["norms"]) - np.array(r64["norms"])) / \
            np.maximum(np.array(r64["norms"]), 1e-300)
        for k in r32["full"]:
            out[f"c3_{mode}_ref32_err_grad:{k}"] = np.float64(rel(r32["full"][k], r64["full"][k]))
        print("c3", mode, "ref fp32 vs fp64: rows", out[f"c3_{mode}_ref32_err_rows"], "norms max",
              float(out[f"c3_{mode}_ref32_err_norms"].max()),
              {k: float(out[f"c3_{mode}_ref32_err_grad:{k}"]) for k in r32["full"]})


def make_c4(out):
    import bench
    from ml3d.torch.models.sparseconvnet import SparseConvUnet
    pos, _ = bench.make_room(0)
    feat = np.random.default_rng(C4_FEAT_SEED).random((len(pos), 3), dtype=np.float32)
    torch.manual_seed(0)
    model = SparseConvUnet(multiplier=32, residual_blocks=True, conv_block_reps=1, num_classes=20,
                           device="cpu").eval()
    sd = model.state_dict()
    model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd))
    inp = types.SimpleNamespace(point=[torch.from_numpy(pos)], feat=[torch.from_numpy(feat)],
                                batch_lengths=[len(pos)])
    t0 = time.time()
    with torch.no_grad():
        logits = model(inp).numpy().astype(np.float32)
    print("c4", logits.shape, round(time.time() - t0, 1), "s", float(np.abs(logits).mean()))
    out["c4_n"] = np.int64(len(pos))
    out["c4_logit_rows"] = logits[::11]
    out["c4_logit_colsum"] = logits.astype(np.float64).sum(0)
    # the same reference model in float64 (same rulebooks; float64 sums): the
    # truth the per-element C4 check holds fp32 results to, and the
    # reference's own fp32 error against it
    import copy
    model64 = copy.deepcopy(model).double()
    inp64 = types.SimpleNamespace(point=[torch.from_numpy(pos).double()], feat=[torch.from_numpy(feat).double()],
                                  batch_lengths=[len(pos)])
    t0 = time.time()
    with torch.no_grad():
        logits64 = model64(inp64).numpy()
    print("c4 f64", round(time.time() - t0, 1), "s")
    out["c4_f64_logit_rows"] = logits64[::11]
    out["c4_ref32_abs_err"] = np.float64(np.abs(logits.astype(np.float64) - logits64).max())
    out["c4_ref32_rel_err"] = np.float64((np.abs(logits.astype(np.float64) - logits64) /
                                          np.maximum(np.abs(logits64), 1e-300)).max())
    print("c4 ref fp32 vs fp64: max abs", float(out["c4_ref32_abs_err"]), "max |f64|", float(np.abs(logits64).max()))


def main():
    import ref_loader
    ref_loader.install()
    out = {}
    parts = sys.argv[1:] or ["c2", "c3", "c4"]
    path = os.path.join(HERE, "full.npz")
    if os.path.exists(path):  # regenerate selected parts only
        old = np.load(path)
        out.update({k: old[k] for k in old.files if k.split("_")[0] not in parts})
    for p in parts:
        {"c2": make_c2, "c3": make_c3, "c4": make_c4}[p](out)
        np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
