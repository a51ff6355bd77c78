"""Generate tests/golden/kpfcnn.npz (build container only): the reference
KPConv collate (ml3d/torch/dataloaders/concat_batcher.py segmentation_inputs
:186-283 with kpconv.py batch_neighbors / batch_grid_subsampling, imported
with tools/ref_loader.py; Open3D's FixedRadiusSearch / ragged_to_dense /
subsample_batch backed by the CPU oracle) and the reference KPFCNN
(kpconv.py:29-291, S3DIS configuration ml3d/configs/kpconv_s3dis.yml scaled
to first_features_dim 32) evaluated with deterministic parameters
(randla_weights.fill) on two small indoor-like clouds.

Stored (data only): the inputs, the random grid rotations the reference drew
(seeded np.random), every layer's points / neighbours / pools / upsamples,
the kernel-point dispositions (the reference's own, from load_kernels —
random fills would put every kernel point out of reach), the eval-mode
logits, loss and the gradients of a few parameters under a cross-entropy
loss, and the same in training mode (batch statistics).  Both are well
conditioned: the reference in fp32 and fp64 agree to ~1e-6 relative."""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402

CFG = dict(lbl_values=list(range(13)), num_classes=13, ignored_label_inds=[], first_subsampling_dl=0.04,
           in_features_dim=5, first_features_dim=32, batch_norm_momentum=0.98, conv_radius=2.5,
           KP_extent=1.2, num_kernel_points=15)
GRAD_KEYS = ["encoder_blocks.0.KPConv.weights", "encoder_blocks.2.unary1.mlp.weight",
             "encoder_blocks.2.KPConv.weights", "encoder_blocks.8.KPConv.weights", "decoder_blocks.1.mlp.weight",
             "head_softmax.mlp.weight"]


def room(n, seed):
    """Points on a floor, two walls and a box inside a 1.6 m room, grid
    subsampled at 0.04 (the cloud segmentation_inputs receives)."""
    import oracle as O
    rng = np.random.default_rng(seed)
    s = rng.integers(0, 4, n)
    u, v = rng.uniform(-0.8, 0.8, (2, n))
    h = rng.uniform(0, 0.02, n)
    p = np.where(s[:, None] == 0, np.stack([u, v, h - 0.8], 1),
                 np.where(s[:, None] == 1, np.stack([u, h - 0.8, v], 1),
                          np.where(s[:, None] == 2, np.stack([h - 0.8, u, v], 1),
                                   np.stack([0.2 + u / 5, 0.3 + v / 5, h - 0.4], 1)))).astype(np.float32)
    return O.subsample(p, sampleDl=0.04)


def batch_inputs():
    a, b = room(6000, 1), room(4000, 2)
    pts = np.concatenate([a, b]).astype(np.float32)
    rng = np.random.default_rng(7)
    feats = np.concatenate([np.ones((len(pts), 1), np.float32), rng.random((len(pts), 4), dtype=np.float32)], 1)
    labels = rng.integers(0, 13, len(pts)).astype(np.int64)
    return pts, feats, labels, np.array([len(a), len(b)], np.int32)


def main():
    import ref_loader
    ref_loader.install()
    os.chdir("/tmp")  # load_kernels writes its kernel dispositions relative to the cwd
    import ml3d.torch.models.kpconv as K
    from ml3d.torch.dataloaders.concat_batcher import KPConvBatch

    pts, feats, labels, lengths = batch_inputs()
    model = K.KPFCNN(**CFG)
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
    li = KPConvBatch.segmentation_inputs(fake, pts, feats, labels, lengths)
    K.create_3D_rotations = orig
    L = cfg.num_layers
    out = {"points": pts, "features": feats, "labels": labels, "lengths": lengths,
           "rotations": np.stack(rots)}
    names = ["layer_points", "neighbors", "pools", "upsamples", "layer_lengths"]
    for gi, name in enumerate(names):
        for l in range(L):
            out[f"{name}_{l}"] = np.asarray(li[gi * L + l]).astype(
                np.float32 if name == "layer_points" else np.int32)
    batch = types.SimpleNamespace(
        points=[torch.from_numpy(li[l]) for l in range(L)],
        neighbors=[torch.from_numpy(li[L + l]) for l in range(L)],
        pools=[torch.from_numpy(li[2 * L + l]) for l in range(L)],
        upsamples=[torch.from_numpy(li[3 * L + l]) for l in range(L)],
        lengths=[torch.from_numpy(li[4 * L + l]) for l in range(L)],
        features=torch.from_numpy(feats), labels=torch.from_numpy(labels))

    sd = model.state_dict()
    keys = list(sd.keys())
    new = randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()], sd)
    for k in keys:
        if k.endswith("kernel_points"):
            new[k] = sd[k].clone()
            out["kp:" + k] = sd[k].numpy().astype(np.float32)
    model.load_state_dict(new)
    model.eval()
    logits = model(batch)
    out["eval_logits"] = logits.detach().numpy().astype(np.float32)
    loss = torch.nn.functional.cross_entropy(logits, batch.labels)
    loss.backward()
    params = dict(model.named_parameters())
    out["eval_loss"] = np.float32(loss.item())
    for k in GRAD_KEYS:
        out["grad_" + k] = params[k].grad.numpy().astype(np.float32)
    model.zero_grad()
    model.train()
    logits = model(batch)
    loss = torch.nn.functional.cross_entropy(logits, batch.labels)
    loss.backward()
    out["train_logits"] = logits.detach().numpy().astype(np.float32)
    out["train_loss"] = np.float32(loss.item())
    for k in GRAD_KEYS:
        out["tgrad_" + k] = params[k].grad.numpy().astype(np.float32)
    out["keys"] = np.array(keys)
    out["shapes"] = np.array([",".join(map(str, sd[k].shape)) for k in keys])
    print("layers", [len(li[l]) for l in range(L)], "nb widths", [li[L + l].shape[1] for l in range(L)],
          "keys", len(keys), "loss", float(loss))
    np.savez_compressed(os.path.join(HERE, "kpfcnn.npz"), **out)


if __name__ == "__main__":
    main()
