"""PointPillars host logic vs the reference (tests/golden/pointpillars.npz,
made by make_golden_pointpillars.py from ml3d/torch/models/point_pillars.py):
identical state_dict keys and shapes (reference checkpoints load unchanged);
the vectorised anchor assignment equals a direct restatement of the
reference's per-target loop (point_pillars.py:826-913); box helpers on known
answers.  Model numerics are checked on the GPU (test_gpu_pointpillars.py)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden_pointpillars import CFG  # noqa: E402

G = np.load(os.path.join(HERE, "golden", "pointpillars.npz"))


def test_state_dict_manifest():
    from o3dml_amd.pointpillars import PointPillars
    sd = PointPillars(**CFG).state_dict()
    assert list(sd.keys()) == [str(k) for k in G["keys"]]
    assert [",".join(map(str, v.shape)) for v in sd.values()] == [str(s) for s in G["shapes"]]


def test_bbox_overlaps_known_answers():
    from o3dml_amd.pointpillars import bbox_overlaps
    a = torch.tensor([[0, 0, 10, 10], [10, 10, 20, 20], [32, 32, 38, 42]], dtype=torch.float32)
    b = torch.tensor([[0, 0, 10, 20], [0, 10, 10, 19], [10, 10, 20, 20]], dtype=torch.float32)
    ref = torch.tensor([[0.5, 0.0, 0.0], [0.0, 0.0, 1.0], [0.0, 0.0, 0.0]])
    assert torch.allclose(bbox_overlaps(a, b), ref)
    assert bbox_overlaps(a[:0], b).shape == (0, 3)


def _loop_assign(head, pred_shape, target_bboxes):
    """point_pillars.py:826-913 restated with its per-target loop."""
    from o3dml_amd.pointpillars import bbox_overlaps, box3d_to_bev2d
    anchors = head.anchor_generator.grid_anchors(pred_shape, device="cpu")
    cnt = int(np.prod(anchors.shape[:-1]))
    rot = anchors.shape[-2]
    outs = [[], [], [], []]
    off = 0
    for i, tb in enumerate(target_bboxes):
        for j, (neg_th, pos_th) in enumerate(head.iou_thr):
            anc = anchors[..., j, :, :].reshape(-1, 7)
            ov = bbox_overlaps(box3d_to_bev2d(tb), box3d_to_bev2d(anc))
            mx, am = ov.max(dim=0)
            gmx, gam = ov.max(dim=1)
            pos = mx >= pos_th
            neg = (mx >= 0) & (mx < neg_th)
            for k in range(len(tb)):
                if gmx[k] >= neg_th:
                    pos[ov[k, :] == gmx[k]] = True
                    am[gam[k]] = k
            outs[0].append(head.bbox_coder.encode(anc[pos], tb[am[pos]]))
            outs[1].append(am[pos] + off)
            f = lambda idx: (idx // rot) * head.num_classes * rot + j * rot + idx % rot + i * cnt  # noqa: E731
            outs[2].append(f(pos.nonzero().squeeze(-1)))
            outs[3].append(f(neg.nonzero().squeeze(-1)))
        off += len(tb)
    return [torch.cat(o, 0) for o in outs]


def test_assign_bboxes_matches_reference_loop():
    from o3dml_amd.pointpillars import PointPillars
    head = PointPillars(**CFG).bbox_head
    tbs = [torch.from_numpy(G[f"bboxes_{i}"]) for i in range(2)]
    # crowd a target pair so several targets compete for the same anchors
    tbs[1] = torch.cat([tbs[1], tbs[1][:2] + torch.tensor([0.05, 0.05, 0, 0, 0, 0, 0.0])])
    pred = torch.zeros((2, 42, 32, 32))
    ours = head.assign_bboxes(pred, tbs)
    ref = _loop_assign(head, (32, 32), tbs)
    for a, b in zip(ours, ref):
        assert a.shape == b.shape and torch.equal(a, b)


def test_dense_loss_equals_indexed_loss():
    """The dense per-anchor loss (no index lists) equals the reference's
    index-list formulation on CPU, including a scene without targets and a
    target of a label outside the classes."""
    from o3dml_amd.pointpillars import PointPillars
    torch.manual_seed(0)
    m = PointPillars(**CFG).eval()
    g = torch.Generator().manual_seed(1)
    out = (torch.randn((3, 18, 32, 32), generator=g), 0.1 * torch.randn((3, 42, 32, 32), generator=g),
           torch.randn((3, 12, 32, 32), generator=g))
    tbs = [torch.from_numpy(G[f"bboxes_{i}"]) for i in range(2)] + [torch.zeros((0, 7))]
    tls = [torch.from_numpy(G[f"labels_{i}"]) for i in range(2)] + [torch.zeros((0,), dtype=torch.long)]
    tls[1] = tls[1].clone()
    tls[1][0] = 3  # not one of the 3 classes
    import types
    inp = types.SimpleNamespace(bboxes=tbs, labels=tls)
    a = m.get_loss(out, inp)
    b = m.get_loss_indexed(out, inp)
    for k in a:
        assert torch.allclose(a[k], b[k], rtol=1e-5, atol=1e-7), (k, a[k], b[k])
