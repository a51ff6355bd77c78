"""Time the reference PointPillars training step on this container's CPU (C5
proxy for DESIGN.md; never shipped): ml3d/torch/models/point_pillars.py with
the pointpillars_kitti.yml model, Open3D voxelize backed by the C oracle
(tools/ref_loader.py), 2 KITTI-shaped scenes (bench.py make_kitti_scene),
AdamW, torch CPU threads = host cores."""
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def main(steps=3):
    import ref_loader
    ref_loader.install()
    import bench
    from ml3d.torch.models.point_pillars import PointPillars
    sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
    from o3dml_amd.pointpillars import DEFAULTS
    torch.manual_seed(0)
    model = PointPillars(device="cpu", augment={}, **DEFAULTS).train()
    opt = torch.optim.AdamW(model.parameters(), lr=0.001, betas=(0.95, 0.99), weight_decay=0.01)
    scenes = [bench.make_kitti_scene(1000 + i) for i in range(2)]
    inp = types.SimpleNamespace(point=[torch.from_numpy(s[0]) for s in scenes],
                                bboxes=[torch.from_numpy(s[1]) for s in scenes],
                                labels=[torch.from_numpy(s[2]) for s in scenes])

    def step():
        t = time.perf_counter()
        loss = sum(model.get_loss(model(inp), inp).values())
        opt.zero_grad()
        loss.backward()
        opt.step()
        return time.perf_counter() - t

    step()
    dt = float(np.median([step() for _ in range(steps)]))
    print(f"reference PointPillars C5 train step (2 scenes) on CPU ({torch.get_num_threads()} threads): "
          f"{dt:.3f} s/step = {2 / dt:.3f} scenes/s")


if __name__ == "__main__":
    main()
