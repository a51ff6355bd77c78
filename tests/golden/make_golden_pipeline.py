"""Generate tests/golden/pipeline.npz (build container only): the reference
RandLA-Net inference pipeline end to end — SemanticSegmentation.run_inference
(ml3d/torch/pipelines/semantic_segmentation.py:122-180) with the
SemSegSpatiallyRegularSampler patch loop (semseg_spatially_regular.py:62-111),
RandLANet.preprocess / transform / update_probs (randlanet.py:115-239,
441-465), imported with tools/ref_loader.py (Open3D ops backed by the C
oracle; sklearn KDTree as in the reference) — on a C2 scan
(bench.make_scan(1), 120,000 points, randlanet_semantickitti.yml model,
deterministic weights from randla_weights.fill, batch_size 1).

The run is seeded (np.random.seed / random.seed before run_inference: the
initial possibilities are the run's first np.random draw and the patch
shuffles its only python-random draws).  Stored, data only: the seeds, the
sub-cloud size, every patch's centre index and the sha256 of its shuffled
index array, the final per-point scores (float16, as the reference stores
them) every 7th row + float64 column sums, and every predicted label."""
import hashlib
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import randla_weights  # noqa: E402

SCAN_SEED = 1
NP_SEED = 123
PY_SEED = 456
NUM_POINTS = 45056


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def main():
    import ref_loader
    ref_loader.install()
    import bench
    from ml3d.datasets.samplers.semseg_spatially_regular import SemSegSpatiallyRegularSampler
    from ml3d.torch.models.randlanet import RandLANet
    from ml3d.torch.pipelines.semantic_segmentation import SemanticSegmentation
    os.chdir("/tmp")
    scan, labels = bench.make_scan(SCAN_SEED)
    torch.manual_seed(0)
    model = RandLANet(num_points=NUM_POINTS, num_classes=19, in_channels=3, augment={"recenter": {"dim": [0, 1]}})
    sd = model.state_dict()
    model.load_state_dict(randla_weights.state_dict_for([(k, tuple(v.shape)) for k, v in sd.items()]))
    centers, shas, sizes = [], [], []
    orig = SemSegSpatiallyRegularSampler.get_point_sampler

    def recording(self):
        gen = orig(self)

        def wrapped(**kw):
            centers.append(int(np.argmin(self.possibilities[self.cloud_id])))
            pc, idxs, center = gen(**kw)
            shas.append(sha(np.asarray(idxs, np.int64)))
            sizes.append(len(idxs))
            return pc, idxs, center
        return wrapped
    SemSegSpatiallyRegularSampler.get_point_sampler = recording
    pipe = SemanticSegmentation(model, dataset=None, device="cpu", batch_size=1, name="SemanticSegmentation",
                                main_log_dir="/tmp/o3dml_logs")
    np.random.seed(NP_SEED)
    random.seed(PY_SEED)
    res = pipe.run_inference({"point": scan, "feat": None, "label": labels})
    SemSegSpatiallyRegularSampler.get_point_sampler = orig
    scores = np.asarray(res["predict_scores"])
    pred = np.asarray(res["predict_labels"])
    print("patches", len(centers), "scores", scores.dtype, scores.shape, "labels", pred.shape)
    out = {"scan_seed": np.int64(SCAN_SEED), "np_seed": np.int64(NP_SEED), "py_seed": np.int64(PY_SEED),
           "num_points": np.int64(NUM_POINTS), "centers": np.array(centers, np.int64), "patch_sha": np.array(shas),
           "patch_sizes": np.array(sizes, np.int64), "score_rows": scores[::7],
           "score_colsum": scores.astype(np.float64).sum(0), "labels": pred.astype(np.int16),
           "n_sub": np.int64(len(pipe.dataset_split.sampler.possibilities[0]))}
    np.savez_compressed(os.path.join(HERE, "pipeline.npz"), **out)
    print("wrote", os.path.getsize(os.path.join(HERE, "pipeline.npz")), "bytes")


if __name__ == "__main__":
    main()
