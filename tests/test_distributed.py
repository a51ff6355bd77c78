"""World-size-2 rehearsal of bench.py's multi-GPU control path on CPU (gloo):
scene sharding by rank (no data-path collective), barrier-bracketed timing and
the max-over-ranks elapsed time every rank agrees on."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time

    import bench
    pts, rs = bench.make_batch(rank, 2, "cpu")
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.02 * (rank + 1))  # rank 1 is the straggler
        return pts.sum()

    elapsed, res = bench.timed_run(step, 5, 2, world, lambda: None)
    q.put((rank, elapsed, len(calls), float(pts[0, 0]), int(rs[-1])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_timing_and_sharding():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, c0, x0, n0), (r1, e1, c1, x1, n1) = out
    assert c0 == c1 == 7  # 2 warmup + exactly 5 timed steps
    assert e0 == e1  # every rank reports the max over ranks
    assert e0 >= 5 * 0.04  # ... which is the straggler's time
    assert x0 != x1  # ranks hold different scenes (seed = rank*100003 + scene)
    assert n0 == n1 == 2 * bench_points()


def bench_points():
    sys.path.insert(0, ROOT)
    import bench
    return bench.N_POINTS


def test_make_batch_is_rank_seeded():
    sys.path.insert(0, ROOT)
    import bench
    a, rs = bench.make_batch(0, 2, "cpu")
    b, _ = bench.make_batch(1, 1, "cpu")
    ref = np.random.default_rng(100003).random((bench.N_POINTS, 3), dtype=np.float32)
    assert torch.equal(b, torch.from_numpy(ref))
    assert a.shape == (2 * bench.N_POINTS, 3) and rs.tolist() == [0, bench.N_POINTS, 2 * bench.N_POINTS]


def _ddp_worker(rank, world, port, q):
    """PointPillars' dense part (SECOND + FPN + anchor head + get_loss) under
    DistributedDataParallel on gloo: after one backward every rank holds the
    average of the per-rank gradients (bench.py pointpillars_bench's C5 path;
    the pillar ops themselves need the GPU)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import types

    from make_golden_pointpillars import CFG
    from o3dml_amd.pointpillars import PointPillars

    class Dense(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.backbone, self.neck, self.bbox_head = m.backbone, m.neck, m.bbox_head

        def forward(self, canvas):
            return self.bbox_head(self.neck(self.backbone(canvas)))

    def batch(r):
        g = torch.Generator().manual_seed(r)
        canvas = torch.relu(torch.randn((1, 64, 64, 64), generator=g))
        boxes = torch.tensor([[3.0 + r, 0.5, -1.7, 1.6, 1.56, 3.9, 0.3], [6.0, -2.0 + r, -0.6, 0.6, 1.73, 0.8, 1.2]])
        return canvas, types.SimpleNamespace(bboxes=[boxes], labels=[torch.tensor([2, 0])])

    grads = []
    for r in range(world):  # single-process reference gradients of every rank's batch
        torch.manual_seed(0)
        m = PointPillars(**CFG).eval()
        canvas, inp = batch(r)
        sum(m.get_loss(Dense(m)(canvas), inp).values()).backward()
        grads.append(torch.cat([p.grad.reshape(-1) for p in Dense(m).parameters()]))
    torch.manual_seed(0)
    m = PointPillars(**CFG).eval()
    ddp = torch.nn.parallel.DistributedDataParallel(Dense(m))
    canvas, inp = batch(rank)
    sum(m.get_loss(ddp(canvas), inp).values()).backward()
    g = torch.cat([p.grad.reshape(-1) for p in ddp.module.parameters()])
    q.put((rank, float((g - sum(grads) / world).abs().max() / (g.abs().max() + 1e-30))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_pointpillars_ddp_gradients():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, err in out:
        assert err < 1e-5


def test_bench_spawns_ranks_without_torchrun():
    """`python bench.py --gpus 2` (no torchrun, WORLD_SIZE unset) starts two
    ranks itself (mp.spawn + env:// rendezvous on 127.0.0.1, as the reference's
    run_pipeline.py:194-206 does); rank 0 prints one line whose value
    aggregates both ranks' units over the max-over-ranks time.  The launcher
    path only (--plumbing-test: gloo on CPU, trivial step)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing-test",
                          "--steps", "3", "--warmup", "1", "--scenes", "2", "--randla-frames", "3"], env=env, capture_output=True,
                         text=True, timeout=240, check=True).stdout
    lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["ranks_reported"] == 2
    assert rec["units_per_rank"] == [2 * 65536 * 3] * 2
    assert abs(rec["value"] - sum(rec["units_per_rank"]) / rec["elapsed_max_s"] / 1e6) < 1e-6 * rec["value"]
    # C2 / C4 legs: --randla-frames scans per rank dealt round-robin, frames over the max time
    shards = rec["scan_shards"]
    assert shards == [[0, 2, 4], [1, 3, 5]]
    assert sorted(sum(shards, [])) == list(range(6))
    assert rec["frames_per_rank"] == [3, 3] and rec["frames_total"] == 6
    if rec["frames_elapsed_max_s"] > 0:
        assert abs(rec["frames_per_s"] - 6 / rec["frames_elapsed_max_s"]) < 1e-6 * rec["frames_per_s"]


def test_shard_round_robin():
    import bench
    for world in (1, 2, 3, 8):
        parts = [bench.shard(13, world, r) for r in range(world)]
        assert sorted(sum(parts, [])) == list(range(13))
        assert all(p == list(range(r, 13, world)) for r, p in enumerate(parts))
    assert bench.shard(6, 1, 0) == list(range(6))  # N = 1: the scans of the single-GPU line
