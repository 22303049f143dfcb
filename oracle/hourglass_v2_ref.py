"""CPU restatement of the CenterNet v2 training path (CenterNet/tf_hourglass_net.py +
CenterNet/train_hourglass_voc.py) — TEST INFRASTRUCTURE ONLY (tests/, smoke, bench cpu_baseline).

  * `format_data` (numpy): the inline target builder of train_hourglass_voc.py train() :96-160 for
    one batch, float32 scalar arithmetic as numpy >= 2 evaluates the reference's expressions
    (np.float32 box rows x Python ints / floats stay float32, NEP 50).  The reference orders boxes
    with np.argsort's default quicksort; on tied areas that order is unspecified, here it is stable.
    Pinned to the reference's own maps (tests/golden/golden_hourglass_v2.npz, made by executing
    train() itself, see make_golden.py).
  * `model_loss` (numpy, float64 from the fp32 inputs): tf_hourglass_net.py:398-413 (focal or
    sigmoid cross-entropy on channels 4.., masked L1 on the sigmoid box channels); pinned to the
    reference's model_loss outputs in the same fixture.
  * `forward` / `loss_and_grads` / `train_step_reference` (torch, autograd): build_model
    (:115-394, separable convs, norm_first BN over sub-batches, bilinear up-sampling, the
    reshape-concat "pass through" of 12 maps, Q36) and train_step (:415-447) with Keras Adam.
    Keras layer semantics restated by hand (TF is absent): conv/BN numerics are parity-unpinned
    at the reference level, as for oracle/centernet_model_ref.py.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .centernet_model_ref import adam_step, bn_group, sepconv, up  # noqa: F401
from .fcos_torch import focal
from .model_ref import _same_pads, q, qg, qw  # noqa: F401

F32 = np.float32


# ---- targets ---------------------------------------------------------------------------------
def format_data(boxes, nbox, raw_dims, img_dims, num_classes):
    """boxes [B][n_max][5] = dataset corner rows (b0, b1, b2, b3) + label (float32); returns the
    reference's img_bbox batch [B][S][S][4][5+C] as float32 (the builder fills float64 arrays with
    float32 values and the step casts them to float32)."""
    B = boxes.shape[0]
    S = img_dims // 8
    out = np.zeros((B, S, S, 4, 5 + num_classes), np.float64)
    pad = int((img_dims - raw_dims) / 2.0)
    scales = [img_dims / (2 ** x) for x in range(4)][::-1]
    for b in range(B):
        bx = np.asarray(boxes[b, :int(nbox[b])], F32)
        xy = (bx[:, :2] + bx[:, 2:4]) / F32(2.0)                 # utils.convert_to_xywh
        wh = bx[:, 2:4] - bx[:, :2]
        area = wh[:, 0] * wh[:, 1] * F32(100)
        for i in np.argsort(area, kind="stable"):
            xc = F32(pad) + xy[i, 0] * F32(raw_dims)
            yc = F32(pad) + xy[i, 1] * F32(raw_dims)
            w = wh[i, 0] * F32(raw_dims)
            h = wh[i, 1] * F32(raw_dims)
            if w < 0 or h < 0:
                continue
            sc = 3
            for k in range(3):
                if w < F32(scales[k]) and h < F32(scales[k]):
                    sc = k
                    break
            bs = F32(scales[sc])
            wc, hc = int(xc / F32(8)), int(yc / F32(8))
            vals = [(yc - F32(hc * 8)) / F32(8), (xc - F32(wc * 8)) / F32(8), h / bs, w / bs]
            if not (-S <= hc < S and -S <= wc < S):
                continue                                          # IndexError in the reference
            out[b, hc, wc, sc, :4] = vals
            out[b, hc, wc, sc, 4] = 1.0
            lab = int(bx[i, 4])
            if 0 <= lab < num_classes:
                out[b, hc, wc, sc, 5 + lab] = 1.0
    return out.astype(F32)


# ---- loss ------------------------------------------------------------------------------------
def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def model_loss(bboxes, logits, b_focal, loss_type="focal"):
    """bboxes [...,4,5+C] targets; logits = the head output BEFORE the model's sigmoid / b_focal
    (the model output is concat(sigmoid(logits[..., :4]), logits[..., 4:] + b_focal)).
    Returns (cls, reg) sums in float64."""
    t = np.asarray(bboxes, np.float64)
    x = np.asarray(logits, F32).astype(np.float64)
    reg = _sig(x[..., :4])
    cls = x[..., 4:] + float(F32(b_focal))
    y = np.trunc(t[..., 4:])
    if loss_type == "sigmoid":
        lc = (np.maximum(cls, 0) - cls * y + np.log1p(np.exp(-np.abs(cls)))).sum()
    else:
        L = np.log1p(np.exp(-np.abs(cls)))
        p = _sig(cls)
        lc = (y * 0.25 * L * (1 - p) ** 2 + p ** 2 * (1 - y) * 0.75 * L
              + (1 - y) * 0.75 * np.maximum(cls, 0) * p ** 2 - y * 0.25 * np.minimum(cls, 0) * (1 - p) ** 2).sum()
    lr = (np.abs(t[..., :4] - reg) * t[..., 4:5]).sum()
    return float(lc), float(lr)


def model_loss_torch(bboxes, logits, b_focal, loss_type="focal"):
    """model_loss with autograd (float64 tensors)."""
    reg = torch.sigmoid(logits[..., :4])
    cls = logits[..., 4:] + b_focal
    y = torch.trunc(bboxes[..., 4:])
    if loss_type == "sigmoid":
        lc = (torch.clamp(cls, min=0) - cls * y + torch.log1p(torch.exp(-cls.abs()))).sum()
    else:
        lc = focal(y, cls)
    lr = ((bboxes[..., :4] - reg).abs() * bboxes[..., 4:5]).sum()
    return lc, lr


# ---- network ---------------------------------------------------------------------------------
def _conv(x, p, name, seperable, stride=1):
    from .centernet_model_ref import dense_conv
    return sepconv(x, p, name, stride=stride) if seperable else dense_conv(x, p, name, stride)


def cnn_block(x, p, blk, group, n_repeats=2, seperable=True, batch_norm=True, norm_order="norm_first"):
    """tf_hourglass_net.cnn_block (:35-77): norm_first (the residual of repeats >= 1 adds the BN
    OUTPUT: tmp_input is rebound to it) or norm_last (BN on the conv output), with / without BN,
    SeparableConv2D or Conv2D."""
    t, res = x, None
    for r in range(n_repeats):
        bn = "%s_bn_%d" % (blk, r)
        if batch_norm and norm_order == "norm_first":
            t = bn_group(t, p, bn, group)
        y = _conv(t, p, "%s_cnn_%d" % (blk, r), seperable)
        if batch_norm and norm_order == "norm_last":
            y = bn_group(y, p, bn, group)
        y = torch.relu(y)
        res = y if r == 0 else q(y + t)
        t = res
    return res


def downsample_block(x, p, name, group, seperable=True, batch_norm=True, norm_order="norm_first"):
    """:79-113: [BN] -> conv 3x3 / 2 ("same") -> [BN] -> ReLU."""
    t = bn_group(x, p, name + "_bnorm", group) if batch_norm and norm_order == "norm_first" else x
    y = _conv(t, p, name, seperable, stride=2)
    if batch_norm and norm_order == "norm_last":
        y = bn_group(y, p, name + "_bnorm", group)
    return torch.relu(y)


def _nhwc(t):
    return t.permute(0, 2, 3, 1)


def forward(x_nhwc, p, num_classes, group, n_repeats=2, seperable=True, batch_norm=True, norm_order="norm_first"):
    """x [B,H,W,3] -> head logits [B,S,S,4,5+C] (before the sigmoid / b_focal), S = H/8."""
    o = dict(seperable=seperable, batch_norm=batch_norm, norm_order=norm_order)
    x = x_nhwc.permute(0, 3, 1, 2)
    B, _, H, W = x.shape
    v = {"blk0": _conv(x, p, "cnn_block_0", seperable)}
    v["cnn1"] = cnn_block(v["blk0"], p, "cnn_block_1", group, n_repeats, **o)
    v["blk1"] = downsample_block(v["cnn1"], p, "down_block_1", group, **o)
    for k in range(2, 7):
        c = cnn_block(v["blk%d" % (k - 1)], p, "cnn_block_%d" % k, group, n_repeats, **o)
        v["in%d" % k] = q(v["blk%d" % (k - 1)] + c)
        v["blk%d" % k] = downsample_block(v["in%d" % k], p, "down_block_%d" % k, group, **o)
    v["dec1"] = cnn_block(q(up(v["blk6"])), p, "dec_block_1", group, n_repeats, **o)
    for k in range(2, 7):
        u = q(up(v["in%d" % (8 - k)] + v["dec%d" % (k - 1)]))
        v["dec%d" % k] = cnn_block(u, p, "dec_block_%d" % k, group, n_repeats, **o)
    S0, S1 = H // 8, W // 8
    order = ["blk1", "blk2", "blk3", "blk4", "blk5", "blk6", "dec1", "dec2", "dec3", "dec4", "dec5", "dec6"]
    feats = torch.cat([_nhwc(v[k]).reshape(B, S0, S1, -1) for k in order], -1).permute(0, 3, 1, 2)
    h = cnn_block(feats, p, "final_out", group, n_repeats, **o)
    w = p["head_out/kernel"]
    out = F.conv2d(F.pad(q(h), (1, 1, 1, 1)), qw(w).permute(3, 2, 0, 1), p["head_out/bias"])
    return qg(_nhwc(out).reshape(B, S0, S1, 4, 5 + num_classes))


def loss_and_grads(params, x, targets, num_classes, sub_batch, loss_type="focal", cls_lambda=2.5, reg_lambda=1.0,
                   **build):
    """train_step's loss over all sub-batches (sums are additive) -> (cls, reg, grads, logits).
    build: forward()'s build options (n_repeats, seperable, batch_norm, norm_order)."""
    p = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    logits = forward(x, p, num_classes, sub_batch, **build)
    lc, lr = model_loss_torch(targets.to(logits.dtype), logits, p["b_focal"], loss_type)
    tot = cls_lambda * lc + reg_lambda * lr
    grads = torch.autograd.grad(tot, list(p.values()), allow_unused=True)
    g = {k: (gg if gg is not None else torch.zeros_like(p[k])) for k, gg in zip(p.keys(), grads)}
    return float(lc), float(lr), g, logits.detach()


def train_step_reference(params, m, v, it, images, targets, num_classes, sub_batch, lr=1e-3, clip=1.0,
                         loss_type="focal"):
    """One tf_hourglass_net.train_step on CPU (in place).  Returns (avg_cls, avg_reg)."""
    B = images.shape[0]
    c, r, g, _ = loss_and_grads(params, images, targets, num_classes, sub_batch, loss_type)
    with torch.no_grad():
        adam_step(params, g, m, v, it, lr, B, clip)
    return c / B, r / B
