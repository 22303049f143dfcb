"""GPU parity of the FCOS inference path (FCOS/infer_fcos.py:27-62): cvl_fcos_detect (corners,
sigmoid scores, combined NMS) vs the numpy restatement oracle/fcos_ref.image_detections.
tf.image.combined_non_max_suppression cannot run here (TF absent): parity is pinned to the
restatement of TF's published kernel, not to TF.  Boxes / classes / valid counts exact, scores
within 4 fp32 ulp (sigmoid evaluation)."""
import numpy as np
import pytest
import torch

from oracle import fcos_ref

pytestmark = pytest.mark.gpu


def _outputs(rng, D, C, strides=(8, 16, 32, 64, 128)):
    """Synthetic FCOS head outputs whose (cell, class) logits are a permutation of an even grid on
    [-18, 6]: no two fp32 scores tie (TF's tie order is unspecified) and neighbouring scores stay
    many ulps apart (the sigmoid is ulp-level unpinned)."""
    shapes = [(-(-D // s), -(-D // s)) for s in strides]
    P = sum(h * w for h, w in shapes)
    logit = (6.0 - rng.permutation(P * C) * (24.0 / (P * C))).reshape(P, C)
    reg = np.concatenate([rng.uniform(-0.5, 4.0, (P, 4)), rng.normal(0, 1, (P, 1))], 1)
    outs, o = [], 0
    for h, w in shapes:
        outs.append(np.concatenate([reg[o:o + h * w], logit[o:o + h * w]], 1).astype(np.float32).reshape(h, w, 5 + C))
        o += h * w
    return outs, shapes


def _fused(outs, C, ld_reg=8, ld_cls=None):
    P = sum(o.shape[0] * o.shape[1] for o in outs)
    ld_cls = ld_cls or C + 3
    reg = np.zeros((P, ld_reg), np.float32)
    cls = np.zeros((P, ld_cls), np.float32)
    o = 0
    for m in outs:
        n = m.shape[0] * m.shape[1]
        reg[o:o + n, :5] = m.reshape(n, -1)[:, :5]
        cls[o:o + n, :C] = m.reshape(n, -1)[:, 5:]
        o += n
    return reg, cls


def _check(got, b, ref):
    bx, sc, cl, nv = ref
    assert int(got.valid_detections[b]) == nv
    np.testing.assert_array_equal(got.nmsed_boxes[b].cpu().numpy(), bx)
    np.testing.assert_array_equal(got.nmsed_classes[b].cpu().numpy(), cl)
    np.testing.assert_allclose(got.nmsed_scores[b].cpu().numpy(), sc, rtol=5e-7, atol=0)


@pytest.mark.parametrize("D,C,center,iou,thr,mpc,tot", [
    (512, 20, False, 0.5, 0.05, 100, 100),     # infer_fcos defaults at the bench geometry
    (512, 20, True, 0.5, 0.05, 100, 100),
    (256, 20, False, 0.3, 0.2, 10, 150),       # per-class cap binds, total not reached
    (128, 80, False, 0.6, 0.5, 50, 40),
    (128, 20, False, 0.5, 0.9999, 100, 100),   # nothing passes: all padding
])
def test_fcos_detect_vs_restatement(D, C, center, iou, thr, mpc, tot):
    from cvlite.infer_fcos import detect_from_outputs
    rng = np.random.default_rng(D + C + int(center))
    B = 2
    imgs = [_outputs(rng, D, C) for _ in range(B)]
    shapes = imgs[0][1]
    fused = [_fused(o, C) for o, _ in imgs]
    reg = torch.tensor(np.stack([f[0] for f in fused])).cuda()
    cls = torch.tensor(np.stack([f[1] for f in fused])).cuda()
    got = detect_from_outputs(reg, cls, shapes, C, center, iou, thr, mpc, tot)
    torch.cuda.synchronize()
    for b in range(B):
        ref = fcos_ref.image_detections(imgs[b][0], C, center, iou, thr, mpc, tot)
        _check(got, b, ref)


def test_fcos_image_detections_model():
    """Model-level path (inference forward with BN running statistics -> detect) vs the oracle on
    the same network outputs."""
    from cvlite import fcos
    from cvlite.infer_fcos import image_detections
    C = 20
    model = fcos.build_model(C)
    rng = np.random.default_rng(4)
    img = rng.uniform(-1, 1, (1, 256, 256, 3)).astype(np.float32)
    got = image_detections(img, model, C, center=False, cls_thresh=0.0101)
    outs = [o[0].cpu().numpy() for o in model(img, training=False)]
    ref = fcos_ref.image_detections(outs, C, False, 0.5, 0.0101, 100, 100)
    assert ref[3] > 0
    _check(got, 0, ref)
