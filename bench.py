#!/usr/bin/env python
"""bench.py — the hot-path benchmark the driver runs (one JSON line on rank 0).

Workload (BASELINE.json metric "Mpoints/s neighbor-search + sparse-conv fwd";
config 1 shape): every GPU holds `--scenes` independent scenes of 65,536
U[0,1)^3 fp32 points (seed = rank*100003 + scene) batched through row splits,
r = 0.05, L2, int32 indices.  One step = the full Open3D
`layers.FixedRadiusSearch` forward on that batch: spatial hash build + count +
scan + host read of the total + fill.  Inputs are resident in HBM before the
timed region.  value = queries processed by all ranks / wall time (Mpoints/s).

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) every rank
is one of its processes; `python bench.py --gpus N` without torchrun spawns
the N processes itself (torch.multiprocessing, 'spawn' start method, before
any GPU call in the parent; rendezvous on 127.0.0.1), mirroring the
reference's mp.spawn + init_process_group (scripts/run_pipeline.py:194-206,
213-251).  Scenes are independent, so there is no data-path collective
("scaling": "weak"); the only collectives are the timing barrier, the
max-over-ranks of the elapsed time and the gather of each rank's processed
units (value = their sum / that time).  The C5 PointPillars leg runs DDP over
RCCL on every rank (its gradient all-reduce is the one real exchange).

roofline: per-kernel HIP-event timing inside the library (events recorded on
the stream each kernel is launched on, o3dml_timing_*); the dominant kernel's
achieved = SURVEY §8d algorithmic bytes (12+12+4+8+4m per query) x queries /
its average duration.  traffic: HBM bytes per launch
from the committed rocprofv3 PMC summary (profiles/), if present.
cpu_baseline: oracle/cpu_frs.c (optimised CPU search of the same semantics, OpenMP,
all host threads and 1 thread) on the bench batch, rank 0, N=1.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "open3d-ml_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N_POINTS = 65536
RADIUS = 0.05



def _fused_opt():
    """Single-kernel (fused) optimizer steps; O3DML_FUSED_OPT=0 for torch's foreach path."""
    return os.environ.get("O3DML_FUSED_OPT", "1") != "0"

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scenes", type=int, default=64, help="C1-shaped scenes per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=5)
    ap.add_argument("--op-reps", type=int, default=20, help="per-op roofline reps: kNN, grid subsample, voxelize "
                    "(0: skip)")
    ap.add_argument("--randla-frames", type=int, default=6, help="RandLA-Net frames timed (0: skip)")
    ap.add_argument("--kpconv-steps", type=int, default=10, help="C3 KPFCNN training steps timed (0: skip)")
    ap.add_argument("--pointpillars-steps", type=int, default=5,
                    help="C5 PointPillars DDP training steps timed on every rank (0: skip)")
    ap.add_argument("--sparse-conv-reps", type=int, default=10, help="C4 sparse-conv forwards timed (0: skip)")
    ap.add_argument("--sweep-reps", type=int, default=5,
                    help="C1 size sweep (one scene of N = 2^16 .. 2^24 pts at constant density): calls timed (0: skip)")
    ap.add_argument("--plumbing-test", action="store_true",
                    help="launcher test only (CPU, gloo): spawn/rendezvous/timing/aggregation with a trivial step "
                         "in place of the GPU workload; reports no metric")
    return ap.parse_args()


def make_batch(rank, scenes, dev):
    pts = np.concatenate([
        np.random.default_rng(rank * 100003 + s).random((N_POINTS, 3), dtype=np.float32)
        for s in range(scenes)])
    rs = np.arange(scenes + 1, dtype=np.int64) * N_POINTS
    return torch.from_numpy(pts).to(dev), torch.from_numpy(rs)


KERNELS = ("frs_group_search", "frs_group_rows")


def c1_sweep(dev, reps):
    """SURVEY §8(d) C1 sweep: one scene of N U[0,1)^3 points, N = 2^16 .. 2^24,
    r = 0.05 (65536/N)^(1/3) (constant neighbour density), one
    layers.FixedRadiusSearch forward per call (hash build + search + fill)."""
    from o3dml_amd import layers
    nns = layers.FixedRadiusSearch()
    out = {}
    for lg in (16, 18, 20, 22, 24):
        n = 1 << lg
        pts = torch.from_numpy(np.random.default_rng(lg).random((n, 3), dtype=np.float32)).to(dev)
        rs = torch.tensor([0, n], dtype=torch.int64)
        r = 0.05 * (65536.0 / n) ** (1.0 / 3.0)
        for _ in range(2):
            res = nns(pts, pts, r, rs, rs)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            res = nns(pts, pts, r, rs, rs)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / reps * 1e3
        pairs = int(res.neighbors_row_splits[-1].item())
        out[str(n)] = {"ms": round(ms, 4), "Mpoints_s": round(n / ms / 1e3, 2), "radius": round(r, 6),
                       "mean_neighbors": round(pairs / n, 3)}
        del pts, res
    torch.cuda.empty_cache()
    return out


def kernel_profile(step, n_queries, pairs, reps):
    """Per-kernel average durations from the library's HIP-event timing (events
    recorded on the stream each kernel is launched on), over `reps` steps."""
    from o3dml_amd import _lib
    lib = _lib.load()
    lib.o3dml_timing_reset()
    lib.o3dml_timing_enable(1)
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    times = _lib.kernel_times(KERNELS)
    lib.o3dml_timing_enable(0)
    avg = {k: (ms / c if c else 0.0) for k, (ms, c) in times.items()}
    dominant = max(avg, key=avg.get)
    mean_nbrs = pairs / n_queries
    alg_bytes = n_queries * (12 + 12 + 4 + 8 + 4 * mean_nbrs)
    return dominant, avg, alg_bytes, mean_nbrs


def load_pmc(kernel):
    """Committed PMC summary of `kernel` (profiles/*/pmc_<kernel>.json written by
    tools/pmc_traffic.py), newest round first; {} when there is none."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_{kernel}.json")), reverse=True):
        try:
            with open(path) as f:
                return json.load(f)
        except Exception:
            continue
    return {}


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary."""
    return load_pmc(kernel).get("hbm_bytes_per_launch")


SIMDS, CLOCK_GHZ, XCDS = 1024, 2.4, 8  # MI355X: 256 CUs x 4 SIMDs in 8 XCDs; 2.4 GHz peak clock
# Measured SIMD issue cost per wave64 VALU instruction at 8 waves per SIMD
# (tools/valu_rate.hip on the box, profiles/r06/valu_rate.jsonl): the search's
# own candidate-test mix (distance, compare into VCC, group mask, mbcnt rank,
# clamped row address, running bcnt count: 17 VALU) issues at 2.62 cycles per
# instruction; v_add_f32 / v_fma_f32 / v_and_b32 alone 2.3, while VOPC into an
# SGPR, v_mbcnt, v_bcnt, v_min_u32, v_lshl_or, v_cndmask and DPP moves are
# ~4.1 each.  (The guide's 4 is ONE wave's issue rate, not the SIMD's.)
VALU_CYC = 2.62
VALU_CYC_SOURCE = "profiles/r06/valu_rate.jsonl (FRS candidate-test mix, 8 waves/SIMD)"


def issue_bound(kernel):
    """How close the search kernel is to its VALU issue ceiling.
    From the committed PMC counters: wave64 VALU instructions x VALU_CYC cycles
    each (measured, see above) over the SIMD-cycles of the measured launch, at the
    clock the same pass ran at (GRBM_GUI_ACTIVE over the 8 XCDs / duration; the
    2.4 GHz peak without it); SALU per CU, 1 cycle each.
    None without a PMC summary."""
    c = load_pmc(kernel).get("counters_per_launch") or {}
    if not c.get("SQ_INSTS_VALU") or not c.get("dur_us_mean"):
        return None
    ghz = c["GRBM_GUI_ACTIVE"] / XCDS / (c["dur_us_mean"] * 1e3) if c.get("GRBM_GUI_ACTIVE") else CLOCK_GHZ
    cyc = c["dur_us_mean"] * 1e3 * ghz
    out = {"valu_instr": int(c["SQ_INSTS_VALU"]), "salu_instr": int(c.get("SQ_INSTS_SALU", 0)),
           "clock_ghz": round(ghz, 3),
           "valu_cyc": VALU_CYC, "valu_cyc_source": VALU_CYC_SOURCE,
           "valu_issue_frac": round(VALU_CYC * c["SQ_INSTS_VALU"] / (SIMDS * cyc), 4),
           "salu_issue_frac": round(c.get("SQ_INSTS_SALU", 0) / (SIMDS / 4 * cyc), 4),
           "source": "profiles/*/pmc_%s.json (PMC pass duration %.1f us)" % (kernel, c["dur_us_mean"])}
    return out


def cpu_baseline(scenes=64):
    """C1 on the host cores, same semantics and output as the GPU step.
    value: oracle/cpu_frs.c (parallel hash build, points in bucket order,
    ONE search pass with AVX2 + FMA candidate tests, block-local outputs
    concatenated) on the bench batch itself (`scenes` x 65,536 points), all
    threads; plus the same code on 1 thread (one scene) and the plain test
    oracle (serial hash build, count + fill passes) for comparison."""
    import oracle as O
    threads = O.default_threads()
    pts, rs = make_batch(0, scenes, "cpu")
    pts, rs = pts.numpy(), rs.numpy()
    one = pts[:N_POINTS]

    def median_rate(fn, n, warm=3, reps=10):  # BASELINE.md timing protocol: 3 warm-ups, median of 10
        for _ in range(warm):
            fn()  # first touch, the oracle build if needed
        times = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            times.append(time.perf_counter() - t)
        return round(n / float(np.median(times)) / 1e6, 4)

    cap = [None, None]

    def fast(p, r, nt, slot):
        idx, _ = O.fixed_radius_search_fast(p, RADIUS, r, nthreads=nt, capacity=cap[slot])
        cap[slot] = len(idx)

    n_thr = median_rate(lambda: fast(pts, rs, threads, 0), len(pts))
    one_thr = median_rate(lambda: fast(one, None, 1, 1), N_POINTS)
    plain = median_rate(lambda: O.fixed_radius_search(one, one, RADIUS, nthreads=threads), N_POINTS)
    return {"value": n_thr, "unit": "Mpoints/s", "cores": threads, "kind": "port",
            "value_1_thread": one_thr, "plain_oracle_value": plain,
            "sample": f"oracle/cpu_frs.c (parallel hash build + one-pass search, AVX2/FMA when the host has "
                      f"them) on the bench batch ({scenes} x 65,536-pt C1 scenes), 3 warm-ups + median of 10, {threads} OpenMP "
                      f"threads; value_1_thread: same code, 1 thread, one scene; plain_oracle_value: the test "
                      f"oracle (serial build, count + fill passes), one scene, {threads} threads"}


def make_scan(seed):
    """C2 synthetic 64-beam scan: elevations -24.8..+2 deg x 1,875
    azimuths = 120,000 rays; ground at z = -1.73 m, one wall per azimuth at
    U(8, 60) m, 2 cm noise, shuffled; labels U{0..19}."""
    rng = np.random.default_rng(seed)
    el = np.deg2rad(np.linspace(-24.8, 2.0, 64))
    az = np.linspace(0, 2 * np.pi, 1875, endpoint=False)
    wall = rng.uniform(8, 60, az.shape[0])
    E, A = np.meshgrid(el, az, indexing="ij")
    W = np.broadcast_to(wall, E.shape)
    r_wall = W / np.cos(E)
    with np.errstate(divide="ignore"):
        r_ground = np.where(E < 0, 1.73 / np.tan(-E), np.inf)
    rr = np.minimum(r_wall, r_ground)
    pts = np.stack([rr * np.cos(E) * np.cos(A), rr * np.cos(E) * np.sin(A), rr * np.sin(E)], -1).reshape(-1, 3)
    pts = pts + rng.normal(0, 0.02, pts.shape)
    pts = pts[rng.permutation(pts.shape[0])].astype(np.float32)
    return pts, rng.integers(0, 20, pts.shape[0]).astype(np.int32)


def shard(n_total, world, rank):
    """Round-robin assignment of n_total independent units (scans, rooms)
    to the ranks: rank r takes units r, r + world, ... (scenes
    shard with no data-path collective)."""
    return list(range(rank, n_total, world))


def frames_over_ranks(frames_local, elapsed_max, world):
    """(all ranks' frames, frames / s over the max-over-ranks time)."""
    counts = gather_units(frames_local, world)
    total = sum(counts)
    return counts, total, (total / elapsed_max if elapsed_max > 0 else 0.0)


def randla_frames(dev, frames, cpu=False, world=1, rank=0):
    """RandLA-Net GPU inference (SemSegInference, randlanet_semantickitti.yml:
    45,056-pt patches, k=16, 4 layers, grid 0.06, random-init weights) on C2
    scans: one frame = the full possibility loop until every sub-point > 0.5.
    `frames` scans per rank (weak scaling), the frames * world scans dealt
    round-robin over the ranks (shard()); at world 1 the scans are seeds
    0 .. frames-1.  Cold pass: each rank's scans once on a fresh model (the
    captured patch graph of every sub-cloud capacity class is built inside
    it); then the timed pass over the same scans (graphs kept per class,
    randlanet._patch_step, as in a stream of scans of similar size).  Both
    passes are bracketed by barrier + device sync, max over ranks."""
    from o3dml_amd.randlanet import RandLANet, SemSegInference
    torch.manual_seed(0)
    model = RandLANet(num_points=45056, num_classes=19).to(dev).eval()
    mine = shard(frames * world, world, rank)
    scans = [torch.from_numpy(make_scan(s)[0]).to(dev) for s in mine]
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731

    def cold():
        for f, sc in enumerate(scans):
            SemSegInference(model, seed=100 + mine[f]).run(sc)

    patches = [0]

    def timed():
        for f, sc in enumerate(scans):
            inf = SemSegInference(model, seed=mine[f])
            inf.run(sc)
            patches[0] += inf.stats["patches"]

    dt_cold, _ = timed_run(cold, 1, 0, world, sync)
    dt, _ = timed_run(timed, 1, 0, world, sync)
    counts, total, fps = frames_over_ranks(len(scans), dt, world)
    _, _, fps_cold = frames_over_ranks(len(scans), dt_cold, world)
    out = {"frames_per_s": round(fps, 3), "ms_per_frame": round(dt / max(len(scans), 1) * 1e3, 2),
           "patches_per_frame": round(patches[0] / max(len(scans), 1), 2), "frames": total, "n_gpus": world,
           "frames_per_rank": counts,
           "cold_frames_per_s": round(fps_cold, 3),
           "cold_ms_per_frame": round(dt_cold / max(len(scans), 1) * 1e3, 2),
           "note": "frames_per_s: scans whose sub-cloud capacity class already has its captured patch graph "
                   "(kept per class); cold_*: the same scans first seen by a fresh model, graph captures included",
           "config": "C2: 120,000-pt synthetic 64-beam scan, RandLANet semantickitti cfg, fp32, random init"
                     + (f", scans round-robin over {world} GPUs" if world > 1 else ""),
           "cpu_reference_s_per_frame_8cores_survey": 10.6}
    if cpu and world == 1:
        out["cpu_baseline"] = randla_cpu_baseline(model, make_scan(0)[0], patches[0] / len(scans))
        out["cpu_baseline"]["gpu_speedup"] = round(out["cpu_baseline"]["value"] / (dt / len(scans)), 1)
    return out


def op_rooflines(dev, reps=20):
    """SURVEY §8(d) per-op rooflines for the ops that dominate C2 / C4 besides
    the FRS search: device time from the library's HIP events (recorded on the
    launch stream around the kernel or phase, o3dml_timing_*), algorithmic
    bytes by §8(d)'s formulas, HBM peak; issue counts from the committed PMC
    summary where one exists (profiles/*/pmc_<kernel>.json).
      knn: the k = 16 self-kNN of one RandLA patch (its 5 levels in one
        batched call, randlanet.py:218-229 <- dataprocessing.py:87-103), the
        search kernel alone; bytes 24 + 4k per query (query xyz, point xyz,
        row split; int32 ids).
      grid_subsample: contrib.subsample of the C2 scan (120,000 pts, dl 0.06;
        randlanet.py:133-139): count + fill phases; bytes per point 12 x 2 +
        8 + 8, per output point 12 + 8.
      voxelize: ops.voxelize of the C4 room at vs = 1 (SparseConvUnet's
        InputLayer, sparseconvnet.py:296-331): count + fill; same formula."""
    from o3dml_amd import _lib, ops
    lib = _lib.load()

    def timed(fn, names):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        lib.o3dml_timing_reset()
        lib.o3dml_timing_enable(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        t = _lib.kernel_times(names)
        lib.o3dml_timing_enable(0)
        return {k: (ms / c if c else 0.0) for k, (ms, c) in t.items()}, e0.elapsed_time(e1) / reps

    def entry(kernel_ms, alg_bytes, call_ms, pmc=None, **extra):
        gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        out = {"bound": "hbm", "kernel_ms": round(kernel_ms, 5), "alg_bytes": int(alg_bytes),
               "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
               "call_ms": round(call_ms, 5)}
        if pmc:
            out["issue"] = issue_bound(pmc)
            out["traffic"] = load_traffic(pmc)
        out.update(extra)
        return out

    res = {}
    scan = torch.from_numpy(make_scan(0)[0]).to(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    center = scan[torch.randint(0, scan.shape[0], (1,), generator=g)]
    d = ((scan - center) ** 2).sum(1)
    lvl = [scan[d.topk(45056, largest=False).indices]]
    for _ in range(4):
        prev = lvl[-1]
        lvl.append(prev[torch.randperm(prev.shape[0], generator=g)[: prev.shape[0] // 4].to(dev)])
    cat = torch.cat(lvl).contiguous()
    krs = torch.tensor(np.cumsum([0] + [x.shape[0] for x in lvl]), dtype=torch.int64)
    m, k = cat.shape[0], 16
    t, call = timed(lambda: ops.knn_search(cat, cat, k, krs, krs), ("knn_search",))
    res["knn"] = entry(t["knn_search"], m * (24 + 4 * k), call, pmc="knn_group",
                       queries=m, k=k, kernel="knn_group_kernel<16, 8, L2>",
                       note="call_ms: the whole knn_search call (grid build, search, row splits, compaction)")
    n = scan.shape[0]
    sub = ops.grid_subsample(scan, [n], 0.06)
    s_n = int(sub[0].shape[0])
    t, call = timed(lambda: ops.grid_subsample(scan, [n], 0.06), ("grid_subsample_count", "grid_subsample_fill"))
    res["grid_subsample"] = entry(t["grid_subsample_count"] + t["grid_subsample_fill"], n * 40 + s_n * 20, call,
                                  points=n, out_points=s_n, dl=0.06,
                                  note="kernel_ms: count + fill phases (keys, segment sort, caps, scan, fill)")
    pos = torch.from_numpy(make_room(0)[0]).to(dev)
    vs = torch.ones(3)
    lo, hi = torch.zeros(3), torch.full((3,), 40960.0)
    vrs = torch.tensor([0, pos.shape[0]], dtype=torch.int64)
    nv = int(ops.voxelize(pos, vrs, vs, lo, hi).voxel_coords.shape[0])
    t, call = timed(lambda: ops.voxelize(pos, vrs, vs, lo, hi), ("voxelize_count", "voxelize_fill"))
    res["voxelize"] = entry(t["voxelize_count"] + t["voxelize_fill"], pos.shape[0] * 40 + nv * 20, call,
                            points=int(pos.shape[0]), voxels=nv,
                            note="kernel_ms: count + fill phases; C4 InputLayer shape")
    return res


def randla_cpu_baseline(model, scan, patches_per_frame, budget_s=30.0):
    """Measured CPU leg of C2 on this host (the reference's
    run_inference on CPU: semseg_spatially_regular.py:79-109, randlanet.py:
    115-239, 441-465): the same RandLANet weights through the model's torch
    path on torch.get_num_threads() cores, grid subsampling by the C oracle
    (OpenMP), every kNN by scipy's cKDTree (workers=-1; the reference uses
    sklearn's KDTree for the crop / projection and nanoflann for the k = 16
    lists).  Sample: one whole frame — the set-up (subsample + 1-NN
    projection) and the patch loop (crop, shuffle, possibility update, 4-level
    kNN, forward, softmax, float16 EMA) until every sub-point's possibility
    exceeds 0.5, the GPU pipeline's stop rule; if the loop outgrows budget_s
    (a slow host), s/frame is extrapolated from the patches done x the GPU
    run's patches per frame, and the sample says so."""
    import oracle as O
    from scipy.spatial import cKDTree
    from o3dml_amd.randlanet import RandLANet
    cpu_model = RandLANet(num_points=45056, num_classes=19)
    cpu_model.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    cpu_model.eval()
    for prm in cpu_model.parameters():
        prm.requires_grad_(False)
    cfg = cpu_model.cfg
    n_pts, k, L = cfg["num_points"], cfg["num_neighbors"], cfg["num_layers"]
    t0 = time.perf_counter()
    sub = O.subsample(scan, sampleDl=cfg["grid_size"])
    tree = cKDTree(sub)
    tree.query(scan, k=1, workers=-1)  # projection of the raw points
    t_setup = time.perf_counter() - t0
    rng = np.random.default_rng(0)
    poss = rng.random(len(sub)) * 1e-3
    probs16 = np.zeros((len(sub), cfg["num_classes"]), np.float16)
    times = []
    while poss.min() <= 0.5 and sum(times) < budget_s:
        t = time.perf_counter()
        cid = int(np.argmin(poss))
        center = sub[cid]
        idx = tree.query(center[None], k=min(n_pts, len(sub)), workers=-1)[1][0]
        rng.shuffle(idx)
        pc = sub[idx].astype(np.float32)
        d = np.sum(np.square(pc - center), 1)
        poss[idx] += np.square(1 - d / np.max(d))
        pc[:, :2] -= center[:2]
        coords, nbrs, subs, ups = [], [], [], []
        cur = pc
        for i in range(L):
            nb = cKDTree(cur).query(cur, k=k, workers=-1)[1]
            nxt = cur[: cur.shape[0] // cfg["sub_sampling_ratio"][i]]
            coords.append(torch.from_numpy(cur)[None])
            nbrs.append(torch.from_numpy(nb)[None])
            subs.append(torch.from_numpy(nb[: nxt.shape[0]])[None])
            ups.append(torch.from_numpy(cKDTree(nxt).query(cur, k=1, workers=-1)[1].reshape(-1, 1))[None])
            cur = nxt
        inputs = {"features": torch.from_numpy(pc)[None], "coords": coords + [torch.from_numpy(cur)[None]],
                  "neighbor_indices": nbrs, "sub_idx": subs, "interp_idx": ups}
        with torch.enable_grad():  # the torch (non-fused) path; no parameter requires grad
            logits = cpu_model(inputs)[0]
        p = torch.softmax(logits, -1).numpy()
        probs16[idx] = probs16[idx] * np.float16(0.95) + np.float32(0.05) * p
        times.append(time.perf_counter() - t)
    t_patch = float(np.mean(times))
    whole = poss.min() > 0.5
    value = t_setup + (sum(times) if whole else patches_per_frame * t_patch)
    how = (f"one whole frame: set-up {t_setup:.2f} s + {len(times)} patches of 45,056 pts ({t_patch:.2f} s "
           f"each) until every possibility > 0.5" if whole else
           f"frame set-up + {len(times)} patches of 45,056 pts ({t_patch:.2f} s each, set-up {t_setup:.2f} s) x "
           f"{patches_per_frame:.2f} patches/frame (the {budget_s:.0f}-s budget ended the loop)")
    return {"value": round(value, 3), "unit": "s/frame", "cores": torch.get_num_threads(), "kind": "port",
            "patches": len(times), "whole_frame": bool(whole), "sample": how}


def make_c3(seed=0, n=20000):
    """C3-shaped KPConv batch: two indoor spheres of radius 1.5 m
    (kpconv_s3dis.yml in_radius) with n points each sampled uniformly on a floor, a
    ceiling and three walls (~25 neighbours at the first conv radius, as on
    0.04-subsampled S3DIS), 5 input features (1, colour + height
    proxies), 13 labels — fed directly to segmentation_inputs."""
    rng = np.random.default_rng(seed)
    clouds = []
    for _ in range(2):
        pts = []
        while sum(len(p) for p in pts) < n:
            m = 4 * n
            s = rng.integers(0, 5, m)
            u, v = rng.uniform(-1.5, 1.5, (2, m))
            h = rng.normal(0, 0.005, m)
            p = np.select([s[:, None] == 0, s[:, None] == 1, s[:, None] == 2, s[:, None] == 3],
                          [np.stack([u, v, h - 0.6], 1), np.stack([u, v, h + 0.7], 1),
                           np.stack([h - 0.5, u, v], 1), np.stack([u, h + 0.6, v], 1)],
                          np.stack([h + 0.8, u, v], 1))
            pts.append(p[np.linalg.norm(p, axis=1) < 1.5])
        clouds.append(np.concatenate(pts)[:n].astype(np.float32))
    pts = np.concatenate(clouds)
    feats = np.concatenate([np.ones((len(pts), 1), np.float32), rng.random((len(pts), 4), dtype=np.float32)], 1)
    return pts, feats, rng.integers(0, 13, len(pts)).astype(np.int64), np.array([n, n], np.int32)


def kpconv_bench(dev, steps):
    """C3: KPFCNN semantic segmentation training step on the GPU, reference
    kpconv_s3dis.yml model (5 layers, K=15, dl0 0.04, first_features_dim 128,
    BN in training mode, random init): GPU collate (segmentation_inputs:
    neighbour searches + grid subsampling per layer) + forward + cross entropy
    + backward + SGD step, ~40k stacked input points per step."""
    from o3dml_amd.kpfcnn import KPFCNN, S3DIS, segmentation_inputs
    blas = os.environ.get("O3DML_BLAS")  # A/B of torch's GEMM backend ("cublas" = rocBLAS, "cublaslt" = hipBLASLt)
    if blas:
        torch.backends.cuda.preferred_blas_library(blas)
    torch.manual_seed(0)
    np.random.seed(0)
    model = KPFCNN(**S3DIS).to(dev).train()
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.98, weight_decay=0.001, fused=_fused_opt())
    pts_np, feat_np, lab_np, lengths = make_c3(0)
    pts = torch.from_numpy(pts_np).to(dev)
    feat = torch.from_numpy(feat_np).to(dev)
    lab = torch.from_numpy(lab_np).to(dev)

    def step():
        batch = segmentation_inputs(model.cfg, pts, feat, lab, lengths)
        loss = model.get_loss(model(batch), batch.labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return batch

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(steps):
        batch = step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t) / steps
    t = time.perf_counter()
    for _ in range(steps):
        segmentation_inputs(model.cfg, pts, feat, lab, lengths)
    torch.cuda.synchronize(dev)
    dt_collate = (time.perf_counter() - t) / steps
    return {"ms_per_step": round(dt * 1e3, 2), "mpoints_per_s": round(len(pts_np) / dt / 1e6, 3),
            "ms_collate": round(dt_collate * 1e3, 2), "layer_points": [int(p.shape[0]) for p in batch.points],
            "neighbor_widths": [int(nb.shape[1]) for nb in batch.neighbors],
            "config": "C3: 2 x 20,000-pt indoor spheres, KPFCNN kpconv_s3dis.yml, fp32, train step "
                      "(GPU collate + fwd + CE + bwd + SGD)"}


def make_kitti_scene(seed, n=20000, n_boxes=10):
    """C5 KITTI-shaped scene: the 64-beam synthetic scan of
    seed `seed` cropped to the camera field of view (|azimuth| < 45 deg) and
    pointpillars_kitti.yml's range [0,69.12] x [-39.68,39.68] x [-3,1], at
    most n points, intensity U[0,1); n_boxes ground-truth boxes (xyzwhlr,
    KITTI class sizes) on the ground with labels 0..2."""
    pts, _ = make_scan(seed)
    keep = (pts[:, 0] > 0) & (np.abs(pts[:, 1]) < pts[:, 0]) & (pts[:, 0] < 69.12) & (np.abs(pts[:, 1]) < 39.68) \
        & (pts[:, 2] > -3) & (pts[:, 2] < 1)
    pts = pts[keep][:n]
    rng = np.random.default_rng(seed + 7)
    pts = np.concatenate([pts, rng.random((len(pts), 1), dtype=np.float32)], 1)
    sizes = ((0.6, 0.8, 1.73), (0.6, 1.76, 1.73), (1.6, 3.9, 1.56))
    labels = rng.integers(0, 3, n_boxes)
    boxes = np.array([[rng.uniform(5, 60), rng.uniform(-25, 25), -1.73, sizes[c][0], sizes[c][2], sizes[c][1],
                       rng.uniform(-np.pi, np.pi)] for c in labels], np.float32)
    return pts.astype(np.float32), boxes, labels.astype(np.int64)


def pointpillars_bench(dev, world, rank, steps, scenes_per_gpu=2):
    """C5: PointPillars (pointpillars_kitti.yml: 3 classes, 432 x 496 pillars,
    random init) training step data-parallel over all ranks: each rank holds
    scenes_per_gpu KITTI-shaped scenes (16 scenes at 8 GPUs); batched GPU
    voxelize + HIP pillar decoration/scatter + SECOND/FPN/head + get_loss +
    backward with the DDP gradient all-reduce over RCCL (bucketed, overlapped
    with backward) + AdamW step."""
    import types
    from o3dml_amd.pointpillars import PointPillars
    torch.manual_seed(0)
    model = PointPillars().to(dev).train()
    ddp = model
    if world > 1:
        ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(model.parameters(), lr=0.001, betas=(0.95, 0.99), weight_decay=0.01, fused=_fused_opt())
    scenes = [make_kitti_scene(1000 + rank * scenes_per_gpu + i) for i in range(scenes_per_gpu)]
    inp = types.SimpleNamespace(point=[torch.from_numpy(s[0]).to(dev) for s in scenes],
                                bboxes=[torch.from_numpy(s[1]).to(dev) for s in scenes],
                                labels=[torch.from_numpy(s[2]).to(dev) for s in scenes])

    def step():
        losses = model.get_loss(ddp(inp), inp)
        loss = sum(losses.values())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    elapsed, _ = timed_run(step, steps, 2, world, lambda: torch.cuda.synchronize(dev))
    n_params = sum(p.numel() for p in model.parameters())
    return {"scenes_per_s": round(world * scenes_per_gpu * steps / elapsed, 3),
            "ms_per_step": round(elapsed / steps * 1e3, 2), "n_gpus": world, "scenes_per_gpu": scenes_per_gpu,
            "global_batch": world * scenes_per_gpu, "points_per_scene": int(scenes[0][0].shape[0]),
            "grad_allreduce_mb": round(n_params * 4 / 2**20, 2) if world > 1 else 0.0,
            "config": "C5: PointPillars pointpillars_kitti.yml train step, KITTI-shaped synthetic scenes, fp32, "
                      + (f"DDP over RCCL x{world}" if world > 1 else "1 GPU")}


def make_room(seed=0):
    """C4-shaped voxel set: ~80k active 2 cm voxels on room surfaces
    (4 m x 3 m floor, 1.2 m walls, four boxes), half-integer positions in voxel
    units in ops.voxelize output order (x-fastest linear id, as InputLayer feeds
    the convolutions), 3 colour features U[0,1)."""
    rng = np.random.default_rng(seed)
    vox = set()
    X, Y, H = 200, 150, 60
    for x in range(X):
        for y in range(Y):
            vox.add((x, y, 0))
    for z in range(H):
        for x in range(X):
            vox.add((x, 0, z)); vox.add((x, Y - 1, z))
        for y in range(Y):
            vox.add((0, y, z)); vox.add((X - 1, y, z))
    for _ in range(4):
        bx, by = rng.integers(20, X - 60), rng.integers(20, Y - 60)
        sx, sy, sz = rng.integers(20, 40, 3)
        for z in range(sz):
            for x in range(bx, bx + sx):
                vox.add((x, by, z)); vox.add((x, by + sy - 1, z))
            for y in range(by, by + sy):
                vox.add((bx, y, z)); vox.add((bx + sx - 1, y, z))
        for x in range(bx, bx + sx):
            for y in range(by, by + sy):
                vox.add((x, y, sz))
    v = np.array(list(vox), np.int64)
    v = v[np.lexsort((v[:, 0], v[:, 1], v[:, 2]))]  # voxelize order: linear id, x fastest
    pos = v.astype(np.float32) + 0.5
    return pos, rng.random((len(pos), 3), dtype=np.float32)


def sparse_conv_bench(dev, reps):
    """C4 submanifold 3^3 sparse convolution, 32 -> 32 channels, fp32 (the
    SparseConvUnet m=32 level-0 conv): full layers.SparseConv forward (rulebook
    via Linf fixed-radius search + kernel index + MFMA gather-GEMM) and the
    GEMM alone (ops.sparse_conv on the prebuilt rulebook)."""
    from o3dml_amd import layers, sparse_conv as sc
    pos_np, _ = make_room(0)
    pos = torch.from_numpy(pos_np).to(dev)
    torch.manual_seed(0)
    conv = layers.SparseConv(32, 32, [3, 3, 3], use_bias=False).to(dev)
    feat = torch.rand((pos.shape[0], 32), device=dev)
    with torch.no_grad():
        out = conv(feat, pos, pos, 1.0)
        nb, kidx = conv._rulebook(pos, pos, 1.0, None, False, 1.0)
        pairs = int(nb.neighbors_index.shape[0])
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(reps):
            out = conv(feat, pos, pos, 1.0)
        torch.cuda.synchronize(dev)
        t_layer = (time.perf_counter() - t) / reps
        t = time.perf_counter()
        for _ in range(reps):
            out = sc.sparse_conv(conv.kernel, feat, None, nb.neighbors_index, kidx, None, nb.neighbors_row_splits)
        torch.cuda.synchronize(dev)
        t_gemm = (time.perf_counter() - t) / reps
    flops = 2.0 * pairs * 32 * 32
    n = pos.shape[0]
    return {"voxels": int(n), "pairs": pairs, "mvoxels_per_s_layer": round(n / t_layer / 1e6, 2),
            "ms_layer": round(t_layer * 1e3, 4), "ms_gemm": round(t_gemm * 1e3, 4),
            "tflops_gemm": round(flops / t_gemm / 1e12, 3),
            "mfma_roofline": [gemm_roofline(dev, pos, nb, kidx, pairs, c, reps, mode)
                              for mode in (1, 0) for c in (32, 128)],
            "config": "C4: ~80k 2 cm room voxels, SparseConv 3^3 32->32 fp32 (exact f32 MFMA products), rulebook rebuilt per call",
            "unet": scn_bench(dev, pos, reps)}


def sparse_conv_ranks(dev, reps, world, rank):
    """N > 1: the C4 SparseConvUnet frames on every rank (rank r's room =
    make_room(r)); the single-GPU layer / GEMM probes run at N = 1 only."""
    pos_np, _ = make_room(rank)
    return {"unet": scn_bench(dev, torch.from_numpy(pos_np).to(dev), reps, world, rank)}


MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense fp32-input MFMA (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA: 256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz
# bf16-split products: useful f32 flop peak = bf16 peak / MFMAs per product
MFMA_SPLIT_PEAK_TFLOPS = {6: round(MFMA_BF16_PEAK_TFLOPS / 6, 1), 3: round(MFMA_BF16_PEAK_TFLOPS / 3, 1)}


def gemm_roofline(dev, pos, nb, kidx, pairs, ch, reps, mode=0):
    """MFMA roofline of the sparse-conv GEMM kernel alone (HIP events around the
    launch inside the library, o3dml_timing_*) on the C4 3^3 map (lattice
    rulebook, cached and tile-ordered as in SparseConvUnet) at ch -> ch
    channels: useful flops 2 * pairs * ch^2 per launch over the kernel time,
    against the MFMA peak of the product precision in use — exact f32-input
    MFMA (mode 1, the default), bf16x6 (mode 0: each f32 operand as hi + mid
    + lo bf16 terms, six bf16 MFMAs per f32 product, peak = bf16 peak / 6) or
    bf16x3 (mode 2, peak = bf16 / 3)."""
    from o3dml_amd import _lib, layers, sparse_conv as sc
    lib = _lib.load()
    prev = lib.o3dml_sparse_conv_set_exact(int(mode))
    try:
        return _gemm_roofline(dev, pos, nb, kidx, pairs, ch, reps, mode)
    finally:
        lib.o3dml_sparse_conv_set_exact(prev)


def _gemm_roofline(dev, pos, nb, kidx, pairs, ch, reps, mode):
    from o3dml_amd import _lib, layers, sparse_conv as sc
    torch.manual_seed(0)
    conv = layers.SparseConv(ch, ch, [3, 3, 3], use_bias=False).to(dev)
    feat = torch.rand((pos.shape[0], ch), device=dev)
    lib = _lib.load()
    with torch.no_grad(), sc.rulebook_cache():  # the map as SparseConvUnet uses it: cached, tile-ordered
        conv(feat, pos, pos, 1.0)
        torch.cuda.synchronize(dev)
        lib.o3dml_timing_reset()
        lib.o3dml_timing_enable(1)
        for _ in range(reps):
            conv(feat, pos, pos, 1.0)
        torch.cuda.synchronize(dev)
        ms, cnt = _lib.kernel_times(["sparse_conv_gemm"])["sparse_conv_gemm"]
        lib.o3dml_timing_enable(0)
    t = ms / max(cnt, 1) / 1e3
    tf = 2.0 * pairs * ch * ch / t / 1e12 if t > 0 else 0.0
    peak = MFMA_F32_PEAK_TFLOPS if mode == 1 else MFMA_SPLIT_PEAK_TFLOPS[6 if mode == 0 else 3]
    return {"channels": ch, "kernel": "implicit_gemm_shared_kernel" if ch >= 64 else "implicit_gemm_lds_kernel",
            "products": {0: "bf16x6", 1: "f32", 2: "bf16x3"}[mode],
            "kernel_us": round(t * 1e6, 2), "bound": "mfma", "achieved": round(tf, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(tf / peak, 4)}


def scn_bench(dev, pos, reps, world=1, rank=0):
    """C4 whole-network forward: SparseConvUnet with the reference scannet
    config (multiplier 32, residual blocks, 1 rep, 20 classes; random init, eval
    mode), InputLayer -> 7-level UNet -> per-point logits, one point per voxel.
    `reps` frames per rank of that rank's room (weak scaling: pos = make_room
    of the rank's seed), bracketed by barrier + device sync, max over ranks."""
    import types
    from o3dml_amd.sparseconvnet import SparseConvUnet
    torch.manual_seed(0)
    m = SparseConvUnet(multiplier=32, residual_blocks=True, conv_block_reps=1, num_classes=20).to(dev).eval()
    feat = torch.rand((pos.shape[0], 3), device=dev)
    inp = types.SimpleNamespace(point=[pos], feat=[feat], batch_lengths=[pos.shape[0]])
    with torch.no_grad():
        # two warmups: the body graph is captured on a size signature's second sighting
        dt, _ = timed_run(lambda: m(inp), reps, 2, world, lambda: torch.cuda.synchronize(dev))
        # the same frames with the body eager (O3DML_SCN_GRAPH=0): the rate of a
        # stream whose scans never repeat a size signature (nothing captured)
        prev = os.environ.get("O3DML_SCN_GRAPH")
        os.environ["O3DML_SCN_GRAPH"] = "0"
        try:
            dt_eager, _ = timed_run(lambda: m(inp), reps, 1, world, lambda: torch.cuda.synchronize(dev))
        finally:
            if prev is None:
                os.environ.pop("O3DML_SCN_GRAPH")
            else:
                os.environ["O3DML_SCN_GRAPH"] = prev
    counts, total, fps = frames_over_ranks(reps, dt, world)
    voxels = sum(gather_units(int(pos.shape[0]) * reps, world))
    return {"ms_per_frame": round(dt / reps * 1e3, 3), "frames_per_s": round(fps, 2),
            "eager_ms_per_frame": round(dt_eager / reps * 1e3, 3),
            "mvoxels_per_s": round(voxels / dt / 1e6, 3), "n_gpus": world, "frames": total,
            "frames_per_rank": counts,
            "config": "SparseConvUnet m=32 residual reps=1 (sparseconvunet_scannet.yml), fp32 (exact f32 MFMA "
                      "products), eval" + (f", one room per GPU x {world}" if world > 1 else "")}


def timed_run(step, steps, warmup, world, sync):
    """W untimed warmups, then EXACTLY `steps` timed steps bracketed by
    barrier + device sync on both sides; returns (max-over-ranks elapsed s,
    last result).  `sync` synchronises the local device (no-op on CPU)."""
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = None
    for _ in range(steps):
        res = step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        backend = dist.get_backend()
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, res


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _spawned(rank, world, port, args):
    """One process per GPU started by `bench.py --gpus N` (no torchrun)."""
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run(args)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import torch.multiprocessing as mp
        mp.spawn(_spawned, args=(args.gpus, _free_port(), args), nprocs=args.gpus, join=True)
        return
    run(args)


def gather_units(units, world):
    """Every rank's processed units (queries) -> list on every rank."""
    if world == 1:
        return [units]
    out = [None] * world
    dist.all_gather_object(out, units)
    return out


def plumbing_test(args, world, rank):
    """Launcher check on CPU (gloo): the same spawn / rendezvous / barrier /
    max-over-ranks / aggregation path as the GPU run, with a trivial CPU step
    in place of the workload.  Reports plumbing fields only, no metric."""
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.ones(1 << 14)
    elapsed, _ = timed_run(lambda: x.sum(), args.steps, args.warmup, world, lambda: None)
    units = gather_units(args.scenes * N_POINTS * args.steps, world)
    # the C2 / C4 legs' sharding: each rank's scans (round-robin) and the
    # frames aggregated over the max-over-ranks time, as randla_frames does
    frames = max(args.randla_frames, 1)
    assigned = gather_units(shard(frames * world, world, rank), world)
    f_elapsed, _ = timed_run(lambda: None, 1, 0, world, lambda: None)
    f_counts, f_total, f_rate = frames_over_ranks(len(assigned[rank]), f_elapsed, world)
    if rank == 0:
        print(json.dumps({"plumbing_test": True, "n_gpus": world, "ranks_reported": len(units),
                          "units_per_rank": units, "value": sum(units) / elapsed / 1e6,
                          "elapsed_max_s": elapsed, "steps": args.steps,
                          "scan_shards": assigned, "frames_per_rank": f_counts, "frames_total": f_total,
                          "frames_elapsed_max_s": f_elapsed, "frames_per_s": f_rate}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing_test:
        return plumbing_test(args, world, rank)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from o3dml_amd import layers
    pts, rs = make_batch(rank, args.scenes, dev)
    nns = layers.FixedRadiusSearch()
    step = lambda: nns(pts, pts, RADIUS, rs, rs)  # noqa: E731
    elapsed, res = timed_run(step, args.steps, args.warmup, world, lambda: torch.cuda.synchronize(dev))
    pairs = int(res.neighbors_row_splits[-1].item())
    units = gather_units(args.scenes * N_POINTS * args.steps, world)

    pp = pointpillars_bench(dev, world, rank, args.pointpillars_steps) if args.pointpillars_steps > 0 else None
    # the sharding workloads run on every rank at N > 1 (collective timing)
    sc_multi = sparse_conv_ranks(dev, args.sparse_conv_reps, world, rank) \
        if world > 1 and args.sparse_conv_reps > 0 else None
    rl_multi = randla_frames(dev, args.randla_frames, False, world, rank) \
        if world > 1 and args.randla_frames > 0 else None
    out = None
    if rank == 0:
        queries_total = sum(units)
        value = queries_total / elapsed / 1e6
        ms_step = elapsed / args.steps * 1e3
        dominant, avg, alg_bytes, mean_nbrs = kernel_profile(step, args.scenes * N_POINTS, pairs, args.kernel_reps)
        ms = avg[dominant]
        achieved = alg_bytes / (ms * 1e-3) / 1e9
        step_achieved = alg_bytes / (ms_step * 1e-3) / 1e9
        out = {
            "metric": "Mpoints/s neighbor-search + sparse-conv fwd; RandLA-Net frames/s",
            "value": round(value, 2),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": "C1 fixed_radius_search: layers.FixedRadiusSearch forward (hash build + search) "
                            f"over {args.scenes} scenes/GPU x 65,536 U[0,1)^3 pts, r=0.05, L2, int32 idx",
                "scenes_per_gpu": args.scenes, "points_per_scene": N_POINTS, "radius": RADIUS,
                "pairs_per_step_rank0": pairs, "parallelism": f"scene-dp{world}",
                "queries_per_rank": units},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(dominant), "kernel_ms": round(ms, 5),
                         "kernel_ms_all": {k: round(v, 5) for k, v in avg.items()},
                         "alg_bytes_per_launch": int(alg_bytes), "mean_neighbors": round(mean_nbrs, 3),
                         "issue": issue_bound(dominant),
                         "step": {"achieved": round(step_achieved, 2), "frac": round(step_achieved / HBM_PEAK_GBS, 4),
                                  "note": "same algorithmic bytes / ms_per_step (hash build, search, "
                                          "row copy and host gaps included)"}},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        if world == 1 and args.sweep_reps > 0:
            out["c1_sweep"] = c1_sweep(dev, args.sweep_reps)
        if world == 1 and args.sparse_conv_reps > 0:
            out["sparse_conv"] = sparse_conv_bench(dev, args.sparse_conv_reps)
        if sc_multi is not None:
            out["sparse_conv"] = sc_multi
        if pp is not None:
            out["pointpillars"] = pp
        if world == 1 and args.kpconv_steps > 0:
            out["kpconv"] = kpconv_bench(dev, args.kpconv_steps)
        if world == 1 and args.randla_frames > 0:
            out["randlanet"] = randla_frames(dev, args.randla_frames, cpu=not args.no_cpu_baseline)
        if world == 1 and args.op_reps > 0:
            ops_rl = op_rooflines(dev, args.op_reps)
            out["ops_roofline"] = ops_rl
            if "randlanet" in out:
                out["randlanet"]["roofline"] = dict(ops_rl["knn"], op="knn (C2 dominant kernel)")
        if rl_multi is not None:
            out["randlanet"] = rl_multi
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
