"""PointPillars C5 train step probe: default NCHW vs channels_last backbone,
per-phase timing (voxelize+PFN+scatter / backbone+neck+head / loss / backward)."""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open3d-ml_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from o3dml_amd.pointpillars import PointPillars  # noqa: E402

dev = torch.device("cuda", 0)
scenes = [bench.make_kitti_scene(1000 + i) for i in range(2)]
inp = types.SimpleNamespace(point=[torch.from_numpy(s[0]).to(dev) for s in scenes],
                            bboxes=[torch.from_numpy(s[1]).to(dev) for s in scenes],
                            labels=[torch.from_numpy(s[2]).to(dev) for s in scenes])
for cl in (False, True, False, True):
    torch.manual_seed(0)
    m = PointPillars().to(dev).train()
    if cl:
        m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.AdamW(m.parameters(), lr=0.001, betas=(0.95, 0.99), weight_decay=0.01)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    tt = [0.0] * 4
    for it in range(13):
        ev[0].record()
        x = m.extract_feats.__self__  # noqa
        with torch.no_grad():
            vox, coors, npts = m.voxel_layer.forward_batch(list(inp.point), decorate=m.voxel_encoder.decoration())
        f = m.voxel_encoder.forward_decorated(vox, npts)
        canvas = m.middle_encoder(f, coors, 2)
        if cl:
            canvas = canvas.contiguous(memory_format=torch.channels_last)
        ev[1].record()
        out = m.bbox_head(m.neck(m.backbone(canvas)))
        ev[2].record()
        loss = sum(m.get_loss(out, inp).values())
        ev[3].record()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        ev[4].record()
        torch.cuda.synchronize()
        if it >= 3:
            for k in range(4):
                tt[k] += ev[k].elapsed_time(ev[k + 1]) / 10
    print("channels_last" if cl else "nchw", " ".join(f"{t:.2f}" for t in tt), f"total {sum(tt):.2f} ms")
