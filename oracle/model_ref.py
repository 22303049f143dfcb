"""torch-CPU restatement of the FCOS ResNet-50-FPN training step (TEST INFRASTRUCTURE and the
bench's `cpu_baseline`).

Restates FCOS/fcos.py:6-110 (graph), Keras ResNet50 v1 (third-party backbone), FCOS/fcos.py:
464-496 (loss, via oracle/fcos_torch.py) and FCOS/train_fcos.py:128-185 (per-image forward, BN
with per-image statistics, sum of per-image gradients, /bs, clip_by_global_norm, Keras SGD).
Parameters are a dict keyed by the Keras layer names used by cvlite's ParamStore.  TF/Keras cannot
run in this image, so these conv/BN numerics are "parity unpinned" at the reference level
(SURVEY.md §8c); they pin the GPU path structurally and numerically.
"""
import math

import torch
import torch.nn.functional as F

from . import fcos_torch

STRIDES = (8, 16, 32, 64, 128)


class _RoundBF16(torch.autograd.Function):
    """Round to bf16 in forward AND round the incoming gradient in backward: places the GPU
    path's bf16 storage points (activations and their gradients) into the fp32 oracle."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class _RoundFwd(torch.autograd.Function):
    """bf16 copy of a weight: rounded forward, fp32 (straight-through) gradient."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """fp32 forward, bf16 gradient (the fused loss writes bf16 head gradients)."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


_EMULATE = {"on": False}


def q(t):
    return _RoundBF16.apply(t) if _EMULATE["on"] else t


def qw(t):
    return _RoundFwd.apply(t) if _EMULATE["on"] else t


def qg(t):
    return _RoundGrad.apply(t) if _EMULATE["on"] else t


class emulate_bf16(object):
    """Context: make the oracle store activations / weights / gradients in bf16 where the GPU
    path does (fp32 arithmetic otherwise).  The FCOS/ResNet-50 graph at random init is chaotic
    (BN nets amplify a per-layer perturbation ~100x over 16 blocks), so an end-to-end bf16-vs-fp32
    comparison measures that amplification, not the kernels; this mode removes it."""

    def __enter__(self):
        _EMULATE["on"] = True

    def __exit__(self, *a):
        _EMULATE["on"] = False


def _same_pads(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def conv(x, p, name, stride=1, pad="same", bias=True):
    """x NCHW; Keras HWIO kernel; TF 'same' (asymmetric for stride 2) or explicit symmetric pad."""
    w = p[name + "/kernel"]
    k = w.shape[0]
    if pad == "same":
        pt, pb = _same_pads(x.shape[2], k, stride)
        pl, pr = _same_pads(x.shape[3], k, stride)
    else:
        pt = pb = pl = pr = int(pad)
    if pt or pb or pl or pr:
        x = F.pad(x, (pl, pr, pt, pb))
    return q(F.conv2d(q(x), qw(w).permute(3, 2, 0, 1), p.get(name + "/bias") if bias else None, stride))


def head_conv(x, p, name):
    """heads write fp32 (no bf16 rounding of the result)."""
    w = p[name + "/kernel"]
    return qg(F.conv2d(F.pad(q(x), (1, 1, 1, 1)), qw(w).permute(3, 2, 0, 1), p[name + "/bias"]))


def bn(x, p, name, eps=1.001e-5):
    """Keras BN in training mode on one image at a time == per-(image, channel) statistics."""
    m = x.mean(dim=(2, 3), keepdim=True)
    v = ((x - m) ** 2).mean(dim=(2, 3), keepdim=True)
    g = p[name + "/gamma"].view(1, -1, 1, 1)
    b = p[name + "/beta"].view(1, -1, 1, 1)
    return (x - m) / torch.sqrt(v + eps) * g + b


def _depths(p):
    """Block counts of conv2_x..conv5_x present in the parameter dict (ResNet50 3/4/6/3,
    ResNet101 3/4/23/3, ResNet152 3/8/36/3 -- Keras applications v1)."""
    out = []
    for st in range(2, 6):
        n = 0
        while "conv%d_block%d_1_conv/kernel" % (st, n + 1) in p:
            n += 1
        out.append(n)
    return tuple(out)


def resnet50(x, p):
    """Keras ResNet50 / 101 / 152 v1 (depth read from the parameter names)."""
    h = conv(x, p, "conv1_conv", 2, pad=3)
    h = q(F.relu(bn(h, p, "conv1_bn")))
    h = F.max_pool2d(F.pad(h, (1, 1, 1, 1)), 3, 2)          # ZeroPadding2D(1) + MaxPool (zeros pad)
    taps = []
    nbs = _depths(p)
    for si, (f, nb, stride) in enumerate(((64, nbs[0], 1), (128, nbs[1], 2), (256, nbs[2], 2), (512, nbs[3], 2))):
        for bi in range(nb):
            n = "conv%d_block%d" % (si + 2, bi + 1)
            s = stride if bi == 0 else 1
            if bi == 0:
                sc = q(bn(conv(h, p, n + "_0_conv", s), p, n + "_0_bn"))
            else:
                sc = h
            y = q(F.relu(bn(conv(h, p, n + "_1_conv", s), p, n + "_1_bn")))
            y = q(F.relu(bn(conv(y, p, n + "_2_conv"), p, n + "_2_bn")))
            y = bn(conv(y, p, n + "_3_conv"), p, n + "_3_bn")
            h = q(F.relu(y + sc))
        taps.append(h)
    return taps[1:]


# Keras MobileNetV2 (alpha 1) blocks 0..16: (expansion, channels, stride)
MBV2_CFG = ((1, 16, 1), (6, 24, 2), (6, 24, 1), (6, 32, 2), (6, 32, 1), (6, 32, 1), (6, 64, 2), (6, 64, 1),
            (6, 64, 1), (6, 64, 1), (6, 96, 1), (6, 96, 1), (6, 96, 1), (6, 160, 2), (6, 160, 1), (6, 160, 1),
            (6, 320, 1))


def mobilenet_v2(x, p):
    """tf.keras.applications.MobileNetV2 (include_top=False) taps block_6_expand, block_13_expand,
    Conv_1 (raw conv outputs; fcos.py:36-41).  BN eps 1e-3 per image, ReLU6, depthwise 3x3 with
    ZeroPadding2D((0,1),(0,1)) + valid at stride 2.  The parameters may carry zero channel pads (the
    cvlite store's layout): zero channels stay zero through every layer, so the result is the
    Keras graph's.  Depthwise kernels are fp32 on the GPU path (no bf16 weight rounding here)."""
    relu6 = lambda t: torch.clamp(t, 0.0, 6.0)  # noqa: E731
    h = q(relu6(bn(conv(x, p, "Conv1", 2, bias=False), p, "bn_Conv1", 1e-3)))
    taps = []
    cin = 32
    for bid, (t, c, s) in enumerate(MBV2_CFG):
        pre = "expanded_conv_" if bid == 0 else "block_%d_" % bid
        res = s == 1 and cin == c
        cin = c
        inp = h
        if t != 1:
            z = conv(h, p, pre + "expand", bias=False)
            if bid in (6, 13):
                taps.append(z)
            h = q(relu6(bn(z, p, pre + "expand_BN", 1e-3)))
        w = p[pre + "depthwise/depthwise_kernel"]
        hp = F.pad(h, (1, 1, 1, 1)) if s == 1 else F.pad(h, (0, 1, 0, 1))
        z = q(F.conv2d(hp, w.permute(2, 3, 0, 1), None, s, groups=w.shape[2]))
        h = q(relu6(bn(z, p, pre + "depthwise_BN", 1e-3)))
        y = bn(conv(h, p, pre + "project", bias=False), p, pre + "project_BN", 1e-3)
        h = q(y + inp) if res else q(y)
    taps.append(conv(h, p, "Conv_1", bias=False))
    return taps


def backbone_taps(x, p):
    return mobilenet_v2(x, p) if "Conv1/kernel" in p else resnet50(x, p)


def fpn_levels(x, p):
    """Backbone + FPN (fcos.py:49-72 == retinanet_module.py:74-105): [P3..P7] NCHW."""
    c3, c4, c5 = backbone_taps(x, p)
    l3 = conv(c3, p, "c3_1x1")
    l4 = conv(c4, p, "c4_1x1")
    l5 = conv(c5, p, "c5_1x1")
    up = lambda t: t.repeat_interleave(2, 2).repeat_interleave(2, 3)  # noqa: E731
    p4r = q(l4 + up(l5))
    p3r = q(l3 + up(l4))
    p6 = conv(c5, p, "c6_3x3", 2)
    return [conv(p3r, p, "c3_3x3"), conv(p4r, p, "c4_3x3"), conv(l5, p, "c5_3x3"), p6,
            conv(F.relu(p6), p, "c7_3x3", 2)]


def fcos_forward(x_nhwc, p, num_classes):
    """Returns reg [B, P, 5] and cls [B, P, C] (level-major cells) like cvlite's FCOSNet."""
    x = x_nhwc.permute(0, 3, 1, 2)
    fpn = fpn_levels(x, p)
    regs, clss = [], []
    for l, f in enumerate(fpn):
        c = f
        r = f
        for i in range(4):
            c = conv(c, p, "cls_layer_%d" % (i + 1), bias=False)
            r = conv(r, p, "reg_layer_%d" % (i + 1), bias=False)
        c = head_conv(F.relu(c), p, "logits_output_%d" % (l + 1))
        r = head_conv(F.relu(r), p, "reg_output_%d" % (l + 1))
        B = x.shape[0]
        clss.append(c.permute(0, 2, 3, 1).reshape(B, -1, num_classes))
        regs.append(r.permute(0, 2, 3, 1).reshape(B, -1, 5))
    return torch.cat(regs, 1), torch.cat(clss, 1)


def fcos_loss_and_grads(params, x, targets, num_classes, grad_scale=1.0, dtype=torch.float32):
    """One batched forward + the reference per-image loss sum; returns losses [B,3] and grads."""
    p = {k: v.detach().to(dtype).requires_grad_(True) for k, v in params.items()}
    reg, cls = fcos_forward(x.to(dtype), p, num_classes)
    tg = targets.to(dtype)
    losses, total = [], 0.0
    for b in range(x.shape[0]):
        lc, lr, le = fcos_torch.packed_loss(reg[b], cls[b], tg[b], num_classes)
        losses.append(torch.stack([lc, lr, le]))
        total = total + (lc + lr + le)
    (total * grad_scale).backward()
    grads = {k: v.grad.detach() for k, v in p.items() if v.grad is not None}
    return torch.stack(losses).detach(), grads, reg.detach(), cls.detach()


def train_step_reference(params, moms, images, targets, num_classes, lr, momentum=0.9, clip=1.0,
                         dtype=torch.float32, losses_out=None):
    """FCOS/train_fcos.py:128-185 restated: per-image forward/backward (batch-1, as the reference),
    gradient sum, /bs, clip_by_global_norm, Keras SGD (v = m v - lr g; w += v).  In place.
    dtype: the arithmetic type (float64 for a tolerance yardstick); losses_out: a list that
    receives each image's (cls, reg, cen) losses (train_fcos.py:157-158)."""
    bs = images.shape[0]
    acc = {k: torch.zeros_like(v) for k, v in params.items()}
    for b in range(bs):
        lo, g, _, _ = fcos_loss_and_grads(params, images[b:b + 1], targets[b:b + 1], num_classes, dtype=dtype)
        if losses_out is not None:
            losses_out.append(lo[0])
        for k, v in g.items():
            acc[k] += v.to(acc[k].dtype)
    for k in acc:
        acc[k] /= bs
    norm = math.sqrt(sum(float((v.double() ** 2).sum()) for v in acc.values()))
    scale = clip / max(norm, clip)
    for k in params:
        g = acc[k] * scale
        moms[k].mul_(momentum).sub_(lr * g)
        params[k].add_(moms[k])
    return norm


def retina_forward(x_nhwc, p, num_classes, n_anchors=9):
    """retinanet_module.py:8-159: shared towers, then per (level, anchor) 3x3 heads.  The params hold
    each level's 9 anchor kernels concatenated on the output axis (`cls_output_{l}` = the Keras
    `cls_output_{l}_anchor_{a}` kernels side by side); returns reg [B, P, 4A] and cls [B, P, AC]
    (level-major cells, anchor a at channels 4a.. / aC..), cvlite's RetinaNetNet layout."""
    x = x_nhwc.permute(0, 3, 1, 2)
    fpn = fpn_levels(x, p)
    regs, clss = [], []
    B = x.shape[0]
    for l, f in enumerate(fpn):
        c = f
        r = f
        for i in range(4):
            c = conv(c, p, "cls_layer_%d" % (i + 1), bias=False)
            r = conv(r, p, "reg_layer_%d" % (i + 1), bias=False)
        c = head_conv(F.relu(c), p, "cls_output_%d" % (l + 1))
        r = head_conv(F.relu(r), p, "reg_output_%d" % (l + 1))
        clss.append(c.permute(0, 2, 3, 1).reshape(B, -1, n_anchors * num_classes))
        regs.append(r.permute(0, 2, 3, 1).reshape(B, -1, n_anchors * 4))
    return torch.cat(regs, 1), torch.cat(clss, 1)


def retina_unpack_targets(tg, level_cells, n_anchors):
    """[B, A*P, 4+C] in (level, anchor, cell) order -> [B, P, A, 4+C] (cell-major, like the preds)."""
    B = tg.shape[0]
    out, o = [], 0
    for S2 in level_cells:
        t = tg[:, o:o + n_anchors * S2].reshape(B, n_anchors, S2, -1).permute(0, 2, 1, 3)
        out.append(t)
        o += n_anchors * S2
    return torch.cat(out, 1)


def retina_loss_and_grads(params, x, targets, num_classes, level_cells, n_anchors=9, img_weight=None,
                          dtype=torch.float32):
    """Forward + RetinaNet.train_loss (retinanet_module.py:403-426: focal over classes, smooth-L1 on
    boxes masked by any class > 0, summed over all levels and anchors) per image; backward of
    sum_b w_b (cls_b + reg_b).  Returns losses [B,2], grads, reg, cls."""
    p = {k: v.detach().to(dtype).requires_grad_(True) for k, v in params.items()}
    reg, cls = retina_forward(x.to(dtype), p, num_classes, n_anchors)
    B, P = reg.shape[0], reg.shape[1]
    t = retina_unpack_targets(targets.to(dtype), level_cells, n_anchors)      # [B, P, A, 4+C]
    losses, total = [], 0.0
    for b in range(B):
        tb = t[b].reshape(P * n_anchors, 4 + num_classes)
        rb = reg[b].reshape(P * n_anchors, 4)
        cb = cls[b].reshape(P * n_anchors, num_classes)
        mask = (tb[:, 4:].max(-1).values > 0).to(tb.dtype)
        lc = fcos_torch.focal(tb[:, 4:], cb)
        lr = fcos_torch.smooth_l1(tb[:, :4], rb, mask)
        w = 1.0 if img_weight is None else float(img_weight[b])
        losses.append(torch.stack([lc, lr]) * w)
        total = total + w * (lc + lr)
    total.backward()
    grads = {k: v.grad.detach() for k, v in p.items() if v.grad is not None}
    return torch.stack(losses).detach(), grads, reg.detach(), cls.detach()
