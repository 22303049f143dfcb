"""CPU restatement of the CenterNet ResNet stride-8 multi-scale path (CenterNet/tf_centernet_resnet_s8.py
with CenterNet/train_centernet_crowdhuman.py) — TEST INFRASTRUCTURE ONLY.

  * `format_data` (numpy, float64 as the reference: its gt_labels are a float32 box array
    concatenated with the int64 class column): :243-330.  np.argsort's quicksort order on tied
    areas is unspecified; here it is stable.  Pinned to the reference's own outputs
    (tests/golden/golden_centernet_s8.npz).
  * `model_loss` (numpy float64 from fp32): :332-385 on the model output (sigmoid'd boxes).
  * `forward` / `loss_and_grads` / `train_step_reference` (torch autograd): build_model :87-208 —
    ResNet C3..C5, 1x1 laterals, P6 = conv3x3/2(P5_1x1) + ReLU, P7, nearest top-down residuals to
    P3, `cnn_feature_map`, the shared 4-layer towers (applied once: every scale reuses the same
    layers on the same input), per-scale 3x3 heads (sigmoid boxes) — and train_step :387-444
    (per-image BN as sub_batch_sz = 1, loss sums, / batch, clip_by_global_norm, Keras SGD
    momentum 0.9).  Keras semantics restated by hand (TF absent): conv / BN numerics parity-unpinned.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .fcos_torch import focal
from .model_ref import conv, q, qg, qw, resnet50  # noqa: F401


# ---- targets ---------------------------------------------------------------------------------
def format_data(gt_labels, box_scales, img_dim, num_classes, img_pad=None, stride=8):
    """gt_labels [n, 5] (y, x, h, w, cls) normalised; returns (float32 [h_max, w_max, ns, 4+C], n)."""
    if img_pad is None:
        img_pad = img_dim
    lab = np.asarray(gt_labels, np.float32).astype(np.float64).reshape(-1, 5)
    h_max, w_max = int(img_pad[1] / stride), int(img_pad[0] / stride)
    pad_y = int((img_pad[1] - img_dim[1]) / 2.0)
    pad_x = int((img_pad[0] - img_dim[0]) / 2.0)
    ns = len(box_scales)
    out = np.zeros((h_max, w_max, ns, num_classes + 4))
    if len(lab) == 0:
        return out.astype(np.float32), 0
    if len(lab) > 1:
        areas = (lab[:, 2] * img_dim[0]) * (lab[:, 3] * img_dim[1])
        lab = lab[np.argsort(areas, kind="stable")]
    for r in lab:
        c = [(r[0] - 0.5 * r[2]) * img_dim[0], (r[1] - 0.5 * r[3]) * img_dim[1],
             (r[0] + 0.5 * r[2]) * img_dim[0], (r[1] + 0.5 * r[3]) * img_dim[1]]
        bh, bw = c[2] - c[0], c[3] - c[1]
        bd = max(bh, bw)
        ok = [s for s in range(ns) if bd < box_scales[s]]
        if not ok:
            continue                                  # ValueError (min of an empty list) there
        sc = min(ok)
        ryc, rxc = (c[0] + c[2]) / 2.0, (c[1] + c[3]) / 2.0
        yc, xc = int((pad_y + ryc) / stride), int((pad_x + rxc) / stride)
        if not (-h_max <= yc < h_max and -w_max <= xc < w_max):
            continue
        out[yc, xc, sc, :4] = [(pad_y + ryc - yc * stride) / stride, (pad_x + rxc - xc * stride) / stride,
                               bh / box_scales[sc], bw / box_scales[sc]]
        k = int(r[4])
        if 0 <= k < num_classes:
            out[yc, xc, sc, 4 + k] = 1.0
    return out.astype(np.float32), len(lab)


# ---- loss ------------------------------------------------------------------------------------
def _focal_np(y, x):
    L = np.log1p(np.exp(-np.abs(x)))
    p = 1.0 / (1.0 + np.exp(-x))
    return (y * 0.25 * L * (1 - p) ** 2 + p ** 2 * (1 - y) * 0.75 * L
            + (1 - y) * 0.75 * np.maximum(x, 0) * p ** 2 - y * 0.25 * np.minimum(x, 0) * (1 - p) ** 2).sum()


def model_loss(y_true, y_pred):
    """:368-385: y_pred [B,S,S,ns,4+C] = (sigmoid boxes, class logits) -> (cls, reg) float64."""
    t = np.asarray(y_true, np.float32).astype(np.float64)
    p = np.asarray(y_pred, np.float32).astype(np.float64)
    mask = (t[..., 4:].max(-1) > 0).astype(np.float64)[..., None]
    d = t[..., :4] - p[..., :4]
    reg = (np.where(np.abs(d) < 1.0, 0.5 * d * d, np.abs(d)) * mask).sum()
    return float(_focal_np(t[..., 4:], p[..., 4:])), float(reg)


def model_loss_torch(y_true, reg_logits, cls_logits):
    """The same on the head logits (sigmoid applied here), autograd."""
    mask = (y_true[..., 4:].max(-1).values > 0).to(reg_logits.dtype).unsqueeze(-1)
    d = y_true[..., :4] - torch.sigmoid(reg_logits)
    reg = (torch.where(d.abs() < 1, 0.5 * d * d, d.abs()) * mask).sum()
    return focal(y_true[..., 4:], cls_logits), reg


# ---- network ---------------------------------------------------------------------------------
def forward(x_nhwc, p, num_classes, n_scales):
    """x [B,H,W,3] -> (reg logits [B,S,S,ns,4], cls logits [B,S,S,ns,C]), S = H/8."""
    x = x_nhwc.permute(0, 3, 1, 2)
    c3, c4, c5 = resnet50(x, p)
    l3, l4, l5 = conv(c3, p, "c3_1x1"), conv(c4, p, "c4_1x1"), conv(c5, p, "c5_1x1")
    p6r = q(F.relu(conv(l5, p, "c6_3x3", 2)))
    p7 = conv(p6r, p, "c7_3x3", 2)
    up = lambda t: t.repeat_interleave(2, 2).repeat_interleave(2, 3)  # noqa: E731  (nearest)
    r6 = q(p6r + up(p7))
    r5 = q(l5 + up(r6))
    r4 = q(l4 + up(r5))
    r3 = q(l3 + up(r4))
    f = conv(r3, p, "cnn_feature_map")
    c, r = f, f
    for i in range(4):
        c = conv(c, p, "cls_layer_%d" % (i + 1), bias=False)
        r = conv(r, p, "reg_layer_%d" % (i + 1), bias=False)
    c, r = q(F.relu(c)), q(F.relu(r))
    B = x.shape[0]
    regs, clss = [], []
    for s in range(n_scales):
        for t, name, out in ((r, "cnn_reg_output_%d", regs), (c, "cnn_cls_output_%d", clss)):
            w = p[name % (s + 1) + "/kernel"]
            o = F.conv2d(F.pad(t, (1, 1, 1, 1)), qw(w).permute(3, 2, 0, 1), p[name % (s + 1) + "/bias"])
            out.append(qg(o.permute(0, 2, 3, 1)).unsqueeze(3))
    return torch.cat(regs, 3), torch.cat(clss, 3)


def loss_and_grads(params, x, targets, num_classes, n_scales, cls_lambda=1.0, reg_lambda=1.0):
    p = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    reg, cls = forward(x, p, num_classes, n_scales)
    lc, lr = model_loss_torch(targets.to(reg.dtype), reg, cls)
    tot = cls_lambda * lc + reg_lambda * lr
    grads = torch.autograd.grad(tot, list(p.values()), allow_unused=True)
    g = {k: (gg if gg is not None else torch.zeros_like(p[k])) for k, gg in zip(p.keys(), grads)}
    return float(lc), float(lr), g, (reg.detach(), cls.detach())


def train_step_reference(params, moms, images, targets, num_classes, n_scales, lr, momentum=0.9, clip=1.0):
    """:387-444 with tf.keras.optimizers.SGD(momentum=0.9) (train_centernet_crowdhuman.py:244):
    per-image BN (sub_batch_sz 1), summed gradients / batch, clip_by_global_norm, v = m v - lr g,
    w += v.  In place; returns (avg_cls, avg_reg)."""
    B = images.shape[0]
    c, r, g, _ = loss_and_grads(params, images, targets, num_classes, n_scales)
    gs = {k: v / B for k, v in g.items()}
    norm = math.sqrt(sum(float((v.double() ** 2).sum()) for v in gs.values()))
    scale = clip / max(norm, clip)
    with torch.no_grad():
        for k in params:
            moms[k].mul_(momentum).sub_(lr * gs[k] * scale)
            params[k].add_(moms[k])
    return c / B, r / B
