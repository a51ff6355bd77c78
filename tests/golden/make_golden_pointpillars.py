"""Generate tests/golden/pointpillars.npz (build container only): the reference
PointPillars (ml3d/torch/models/point_pillars.py, imported with
tools/ref_loader.py; Open3D's voxelize / ragged_to_dense backed by the CPU
oracle) with the pointpillars_kitti.yml architecture on a reduced 10.24 m x
10.24 m range (64 x 64 pillars) so the fixture stays small, deterministic
parameters (randla_weights.fill), two synthetic LiDAR-like scenes with
ground-truth boxes of the three KITTI classes.

Stored (data only): inputs, the first scene's voxelization, eval-mode head
outputs, and for one forward + get_loss + backward in eval mode (running
batch-norm statistics: well conditioned, the reference in fp32 and fp64
agree to <1e-6) and in training mode (batch statistics over 32 x 32 .. 8 x 8
maps: fp32 and fp64 differ by up to 0.7% in the backbone gradients) the
three losses and a few parameter gradients.

`--full` writes tests/golden/pointpillars_full.npz instead: the reference
config itself (ml3d/configs/pointpillars_kitti.yml model section: 432 x 496
pillars over [0, 69.12] x [-39.68, 39.68], max_voxels 16000 / 40000) on the
two KITTI-shaped scenes bench.py's C5 leg times on rank 0
(bench.make_kitti_scene(1000), (1001)): scene 0's voxelization, eval-mode
head outputs (float64 per-channel sums plus 4,096 sampled entries per
output, the full maps are ~30 MB), and per mode the losses and GRAD_KEYS
gradients.  The same forward / loss / backward is also run on the
reference in float64 (model, points and the decorated pillars in double)
and the fp32-vs-fp64 spread of every stored value is recorded, so the test
tolerances are the reference's own precision at this size."""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402

RANGE = [0, -5.12, -3, 10.24, 5.12, 1]
CFG = dict(
    point_cloud_range=RANGE, classes=["Pedestrian", "Cyclist", "Car"],
    voxelize=dict(max_num_points=32, voxel_size=[0.16, 0.16, 4], max_voxels=[16000, 40000]),
    voxel_encoder=dict(in_channels=4, feat_channels=[64], voxel_size=[0.16, 0.16, 4]),
    scatter=dict(in_channels=64, output_shape=[64, 64]),
    head=dict(in_channels=384, feat_channels=384, nms_pre=100, score_thr=0.1,
              ranges=[[0, -5.12, -0.6, 10.24, 5.12, -0.6], [0, -5.12, -0.6, 10.24, 5.12, -0.6],
                      [0, -5.12, -1.78, 10.24, 5.12, -1.78]],
              sizes=[[0.6, 0.8, 1.73], [0.6, 1.76, 1.73], [1.6, 3.9, 1.56]], rotations=[0, 1.57],
              iou_thr=[[0.35, 0.5], [0.35, 0.5], [0.45, 0.6]]),
    loss=dict(focal=dict(gamma=2.0, alpha=0.25, loss_weight=1.0), smooth_l1=dict(beta=0.11, loss_weight=2.0),
              cross_entropy=dict(loss_weight=0.2)))
GRAD_KEYS = ["voxel_encoder.pfn_layers.0.linear.weight", "backbone.blocks.0.0.weight", "backbone.blocks.1.3.weight",
             "neck.deblocks.1.0.weight", "bbox_head.conv_cls.weight", "bbox_head.conv_reg.weight",
             "bbox_head.conv_dir_cls.weight"]


def scene(seed, n=3000, n_boxes=5):
    """Ground returns + points on box-shaped objects inside RANGE, intensity
    U[0,1); boxes xyzwhlr (KITTI bottom-centre z) with labels 0..2."""
    rng = np.random.default_rng(seed)
    g = np.stack([rng.uniform(0, 10.2, n), rng.uniform(-5.1, 5.1, n), rng.normal(-1.7, 0.03, n)], 1)
    sizes = {0: (0.6, 0.8, 1.73), 1: (0.6, 1.76, 1.73), 2: (1.6, 3.9, 1.56)}
    boxes, labels, obj = [], [], []
    for _ in range(n_boxes):
        c = int(rng.integers(0, 3))
        w, l, h = sizes[c]
        x, y, yaw = rng.uniform(1.5, 9), rng.uniform(-4, 4), rng.uniform(-np.pi, np.pi)
        boxes.append([x, y, -1.7, w, h, l, yaw])
        labels.append(c)
        m = 300
        u = rng.uniform(-0.5, 0.5, (m, 3)) * [l, w, h]
        R = np.array([[np.cos(yaw), -np.sin(yaw)], [np.sin(yaw), np.cos(yaw)]])
        xy = u[:, :2] @ R.T + [x, y]
        obj.append(np.concatenate([xy, u[:, 2:] + h / 2 - 1.7], 1))
    pts = np.concatenate([g] + obj).astype(np.float32)
    pts = np.concatenate([pts, rng.random((len(pts), 1), dtype=np.float32)], 1)
    return pts[rng.permutation(len(pts))], np.array(boxes, np.float32), np.array(labels, np.int64)


def full_cfg():
    """The model section of the reference's pointpillars_kitti.yml (no augmentation)."""
    import yaml
    with open("/root/reference/ml3d/configs/pointpillars_kitti.yml") as f:
        m = yaml.safe_load(f)["model"]
    keep = ("point_cloud_range", "classes", "loss", "voxelize", "voxel_encoder", "scatter", "backbone", "neck",
            "head")
    return {k: m[k] for k in keep}


SAMPLE = 4096  # sampled entries per head output in the full fixture


def main_full():
    import ref_loader
    ref_loader.install()
    sys.path.insert(0, ROOT)
    import bench
    from ml3d.torch.models.point_pillars import PointPillars

    cfg = full_cfg()
    scenes = [bench.make_kitti_scene(1000 + i) for i in range(2)]
    torch.manual_seed(0)
    model = PointPillars(device="cpu", augment={}, **cfg)
    sd = model.state_dict()
    model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd))
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    inputs = types.SimpleNamespace(point=[torch.from_numpy(s[0]) for s in scenes],
                                   bboxes=[torch.from_numpy(s[1]) for s in scenes],
                                   labels=[torch.from_numpy(s[2]) for s in scenes])
    out = {}
    for i, (p, b, l) in enumerate(scenes):
        out[f"points_{i}"], out[f"bboxes_{i}"], out[f"labels_{i}"] = p, b, l
    rng = np.random.default_rng(0)

    def run(m, dtype):
        """eval head outputs, then per mode losses + GRAD_KEYS grads, in dtype."""
        res = {}
        m.load_state_dict(sd0)  # the train-mode pass below moves the BN running statistics
        m = m.to(dtype)
        if dtype == torch.float64:  # decorated pillars in double too (the voxelizer's ids are exact)
            enc = m.voxel_encoder
            f32_fwd = enc.forward

            def fwd(features, num_points, coors):
                return f32_fwd(features.double(), num_points, coors)
            enc.forward = fwd
        m.eval()
        with torch.no_grad():
            heads = m(inputs)
        for name, t in zip(("cls", "reg", "dir"), heads):
            res[f"eval_{name}"] = t.double().numpy()
        params = dict(m.named_parameters())
        for mode in ("eval", "train"):
            m.zero_grad()
            m.train(mode == "train")
            r = m(inputs)
            losses = m.get_loss(r, inputs)
            sum(losses.values()).backward()
            for k, val in losses.items():
                res[f"{mode}_{k}"] = float(val.item())
            for k in GRAD_KEYS:
                res[f"{mode}_grad_{k}"] = params[k].grad.double().numpy()
        return res

    m32 = run(model, torch.float32)
    model.eval()
    with torch.no_grad():
        v, c, n = model.voxel_layer(inputs.point[0])
    out["vox_coords_0"], out["vox_num_0"] = c.numpy(), n.numpy()
    out["vox_sum_0"] = v.double().sum(dim=(1, 2)).numpy()
    m64 = run(model, torch.float64)
    spread = {}
    for k, a in m32.items():
        b = m64[k]
        if k in ("eval_cls", "eval_reg", "eval_dir"):
            flat = a.reshape(-1)
            sel = rng.choice(flat.size, SAMPLE, replace=False)
            out[f"{k}_shape"] = np.array(a.shape)
            out[f"{k}_sel"] = sel.astype(np.int64)
            out[f"{k}_val"] = flat[sel].astype(np.float32)
            out[f"{k}_chsum"] = a.sum(axis=(0, 2, 3))
            out[f"{k}_chabs"] = np.abs(a).sum(axis=(0, 2, 3))
            spread[k] = float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))
        elif isinstance(a, np.ndarray):
            out[k] = a.astype(np.float32)
            spread[k] = float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))
        else:
            out[k] = np.float64(a)
            spread[k] = abs(a - b) / (abs(b) + 1e-30)
    out["spread_keys"] = np.array(list(spread))
    out["spread_vals"] = np.array([spread[k] for k in spread], np.float64)
    print("voxels", v.shape, {k: f"{x:.2e}" for k, x in spread.items()})
    np.savez_compressed(os.path.join(HERE, "pointpillars_full.npz"), **out)


def main():
    import ref_loader
    ref_loader.install()
    from ml3d.torch.models.point_pillars import PointPillars

    scenes = [scene(s) for s in (0, 1)]
    torch.manual_seed(0)
    model = PointPillars(device="cpu", augment={}, **CFG)
    sd = model.state_dict()
    keys = list(sd.keys())
    model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd))
    inputs = types.SimpleNamespace(point=[torch.from_numpy(s[0]) for s in scenes],
                                   bboxes=[torch.from_numpy(s[1]) for s in scenes],
                                   labels=[torch.from_numpy(s[2]) for s in scenes])
    out = {}
    for i, (p, b, l) in enumerate(scenes):
        out[f"points_{i}"], out[f"bboxes_{i}"], out[f"labels_{i}"] = p, b, l
    model.eval()
    with torch.no_grad():
        v, c, n = model.voxel_layer(inputs.point[0])
        out["vox_coords_0"], out["vox_num_0"] = c.numpy(), n.numpy()
        out["vox_sum_0"] = v.double().sum(dim=(1, 2)).numpy()
        cls, reg, dr = model(inputs)
    out["eval_cls"], out["eval_reg"], out["eval_dir"] = cls.numpy(), reg.numpy(), dr.numpy()
    params = dict(model.named_parameters())
    for mode in ("eval", "train"):
        model.zero_grad()
        model.train(mode == "train")
        res = model(inputs)
        losses = model.get_loss(res, inputs)
        sum(losses.values()).backward()
        for k, val in losses.items():
            out[f"{mode}_{k}"] = np.float32(val.item())
        for k in GRAD_KEYS:
            out[f"{mode}_grad_{k}"] = params[k].grad.numpy().astype(np.float32)
    out["keys"] = np.array(keys)
    out["shapes"] = np.array([",".join(map(str, sd[k].shape)) for k in keys])
    print("voxels", v.shape, "keys", len(keys), {k: float(x) for k, x in losses.items()})
    np.savez_compressed(os.path.join(HERE, "pointpillars.npz"), **out)


if __name__ == "__main__":
    if "--full" in sys.argv[1:]:
        main_full()
    else:
        main()
