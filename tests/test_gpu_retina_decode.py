"""GPU parity of the RetinaNet inference decode (retinanet_module.py:428-529): cvl_retina_corners
and cvl_retina_nms bit-exact vs the reference's goldens; cvl_retina_decode + NMS vs the goldens
(boxes / labels / kept rows exact, scores within 4 fp32 ulp: the sigmoid is ulp-level unpinned) and
vs the oracle at full 640x640 COCO size, batched, plus the model-level image_detections path."""
import numpy as np
import pytest
import torch

from oracle import retina_ref

pytestmark = pytest.mark.gpu


def _fused(outs_levels, C):
    """nested [5][A] arrays [S,S,4+C] (one image) -> fused head layout reg [P, 4A], cls [P, A*C]."""
    regs, clss, shapes = [], [], []
    for lev in outs_levels:
        S0, S1 = lev[0].shape[:2]
        shapes.append((S0, S1))
        regs.append(np.concatenate([m[..., :4].reshape(-1, 4) for m in lev], 1))
        clss.append(np.concatenate([m[..., 4:].reshape(-1, C) for m in lev], 1))
    return np.concatenate(regs, 0), np.concatenate(clss, 0), shapes


def _net(C):
    from cvlite.retinanet import RetinaNet
    return RetinaNet(C, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])


def _compare(got, ref):
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(got[:, [0, 1, 2, 3, 5]], ref[:, [0, 1, 2, 3, 5]])
    np.testing.assert_allclose(got[:, 4], ref[:, 4], rtol=5e-7, atol=0)


def test_retina_corners_and_nms_bit_exact(golden):
    d = golden("retina_decode")
    net = _net(80)
    np.testing.assert_array_equal(net.prediction_to_corners(d["corners_in"], d["corners_dims"], 32), d["corners_out"])
    np.testing.assert_array_equal(net.cpu_nms(d["nms_dets"], 0.45), d["nms_keep"])
    assert len(net.cpu_nms(np.zeros((0, 6), np.float32), 0.5)) == 0


def test_retina_decode_matches_reference_goldens(golden):
    d = golden("retina_decode")
    i = 0
    while "case_%d_cfg" % i in d:
        D, C, iou_t, cls_t = d["case_%d_cfg" % i]
        C = int(C)
        net = _net(C)
        np.testing.assert_array_equal(np.array(net.anchor_boxes, np.float32), d["case_%d_anchor_dims" % i])
        outs = [list(d["case_%d_out_L%d" % (i, l)]) for l in range(5)]
        reg, cls, shapes = _fused(outs, C)
        # pad the rows to the model's channel pitch (ld > 4A / AC) to exercise the strides
        regp = np.zeros((1, reg.shape[0], 4 * 9 + 28), np.float32)
        clsp = np.zeros((1, cls.shape[0], 9 * C + 3), np.float32)
        regp[0, :, :36] = reg
        clsp[0, :, :9 * C] = cls
        got = net.decode_detections(torch.tensor(regp).cuda(), torch.tensor(clsp).cuda(), shapes,
                                    iou_thresh=float(iou_t), cls_thresh=float(cls_t))[0]
        _compare(got, d["case_%d_dets" % i])
        i += 1
    assert i == 4


def _synthetic_outputs(rng, D, C, strides=(8, 16, 32, 64, 128)):
    S = [D // s for s in strides]
    R = 9 * sum(x * x for x in S)
    win = (rng.permutation(R) - 0.8 * R) / 2048.0
    outs, o = [], 0
    for l in range(5):
        lev = []
        for a in range(9):
            n = S[l] * S[l]
            reg = np.concatenate([rng.normal(0, 0.5, (n, 2)), rng.uniform(0.3, 2.5, (n, 2))], 1)
            cls = win[o:o + n, None] - rng.uniform(0.5, 6.0, (n, C))
            cls[np.arange(n), rng.integers(0, C, n)] = win[o:o + n]
            o += n
            lev.append(np.concatenate([reg, cls], 1).astype(np.float32).reshape(S[l], S[l], 4 + C))
        outs.append(lev)
    return outs


def test_retina_decode_batched_full_size_vs_oracle():
    """configs[4] geometry: 640x640, COCO C=80, 76,725 anchors per image, B=2."""
    rng = np.random.default_rng(5)
    C, D, B = 80, 640, 2
    net = _net(C)
    dims = np.array(net.anchor_boxes, np.float32)
    imgs = [_synthetic_outputs(rng, D, C) for _ in range(B)]
    fused = [_fused(o, C) for o in imgs]
    reg = torch.tensor(np.stack([f[0] for f in fused])).cuda()
    cls = torch.tensor(np.stack([f[1] for f in fused])).cuda()
    got = net.decode_detections(reg, cls, fused[0][2], iou_thresh=0.5, cls_thresh=0.3)
    for b in range(B):
        ref = retina_ref.image_detections(imgs[b], dims, iou_thresh=0.5, cls_thresh=0.3)
        assert len(ref) > 100
        _compare(got[b], ref)


def test_retina_image_detections_model():
    """The model-level path: inference forward (BN running stats) -> decode -> NMS, checked
    against the oracle applied to the same network outputs."""
    net = _net(20)
    rng = np.random.default_rng(3)
    img = rng.uniform(-1, 1, (1, 256, 256, 3)).astype(np.float32)
    dets = net.image_detections(img, iou_thresh=0.5, cls_thresh=0.0101)
    m = net.model
    x = torch.tensor(img).cuda()
    shapes, _, _ = m.layout(1, 256, 256)
    reg, cls = m.forward(x, train=False)
    nested = m.outputs_nested(reg, cls, 256, 256)
    outs = [[t[0].cpu().numpy() for t in lev] for lev in nested]
    ref = retina_ref.image_detections(outs, np.array(net.anchor_boxes, np.float32), iou_thresh=0.5,
                                      cls_thresh=0.0101)
    _compare(dets, ref)
