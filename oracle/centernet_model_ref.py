"""torch-CPU restatement of the CenterNet hourglass training step — TEST INFRASTRUCTURE and the
CenterNet bench line's `cpu_baseline`.

Restates CenterNet/tf_centernet_hourglass.py:
  * `cnn_block` (:87-156): per repeat [BN (norm_first) -> SeparableConv 1x1 (n_filters) ->
    SeparableConv kxk (n_filters) -> SeparableConv 1x1 (2*n_filters) -> ReLU]; from the second
    repeat on, the residual adds `tmp_input`, which at that point is the BN OUTPUT (:103-106,
    :150-155 — the input is rebound to the normalised tensor);
  * `downsample_block` (:158-161) MaxPooling2D(2, 2, "same");
  * `build_model` (:163-353): SeparableConv 7x7/2 stem, cnn_block_1, max_pool_1, one hourglass
    stack (4 encoder blocks with residual + pool, 4 decoder merges with bilinear x2 up-sampling),
    3x3 `cnn_out` conv (4+C), `b_focal` BiasLayer on the class channels (:345-350);
  * `model_loss` / `focal_loss` / `smooth_l1_loss` (:458-505);
  * `train_step` (:507-564): one training-mode forward per sub-batch (BN statistics over the
    sub-batch), loss = 2.5 cls + 1.0 reg, gradients summed over sub-batches then / batch_size,
    clip_by_global_norm, optimizer (Keras Adam, train_hourglass_voc.py:330).
Keras layer semantics restated by hand (TF absent here): SeparableConv2D =
depthwise (depth_multiplier 1, no bias) then pointwise + bias; TF "same" padding; BN eps 1e-3,
momentum 0.99; UpSampling2D(bilinear) = resize_bilinear with half-pixel centres (= torch
bilinear, align_corners=False).  Conv/BN numerics are "parity unpinned" at the reference level.
"""
import math

import torch
import torch.nn.functional as F

from .model_ref import _same_pads, emulate_bf16, q, qg, qw  # noqa: F401  (bf16-storage emulation)
from .fcos_torch import focal

BN_EPS = 1e-3


def blocks(n_stacks=1):
    """(name, input, output) of every cnn_block in graph order (tf_centernet_hourglass.py:189-333)."""
    out = [("cnn_block_1", "blk0", "cnn1")]
    for s in range(n_stacks):
        st = "stack_%d_" % (s + 1)
        out += [(st + "enc_block_1", "stack_in", "enc1"), (st + "enc_block_2", "e1", "enc2"),
                (st + "enc_block_3", "e2", "enc3"), (st + "enc_block_4a", "e3", "enc4a"),
                (st + "enc_block_4b", "enc4a", "enc4b"), (st + "enc_block_4", "enc4b", "enc4"),
                (st + "dec_block_1", "e3", "dec1"), (st + "dec_out_1", "d1res", "o1"),
                (st + "dec_block_2", "e2", "dec2"), (st + "dec_out_2", "d2res", "o2"),
                (st + "dec_block_3", "e1", "dec3"), (st + "dec_out_3", "d3res", "o3"),
                (st + "dec_block_4", "stack_in", "dec4"), (st + "dec_out_4", "d4res", "o4")]
    return out


def sepconv(x, p, name, stride=1):
    """Keras SeparableConv2D, x NCHW.  fp32: depthwise then pointwise (the reference's order);
    bf16 emulation: the GPU path's folded dense kernel D*P on bf16 operands."""
    dw, pw, b = p[name + "/depthwise_kernel"], p[name + "/pointwise_kernel"], p[name + "/bias"]
    k, C = dw.shape[0], dw.shape[2]
    pt, pb = _same_pads(x.shape[2], k, stride)
    pl, pr = _same_pads(x.shape[3], k, stride)
    xp = F.pad(x, (pl, pr, pt, pb)) if (pt or pb or pl or pr) else x
    from .model_ref import _EMULATE
    if _EMULATE["on"]:
        weff = dw[..., 0].unsqueeze(-1) * pw[0, 0].unsqueeze(0).unsqueeze(0)     # [k,k,C,Cout]
        return q(F.conv2d(q(xp), qw(weff).permute(3, 2, 0, 1), b, stride))
    y = F.conv2d(xp, dw.permute(2, 3, 0, 1), None, stride, groups=C)
    return F.conv2d(y, pw.permute(3, 2, 0, 1), b)


def dense_conv(x, p, name, stride=1):
    """Keras Conv2D(..., padding="same") with bias (build_model(seperable=False), :124-136)."""
    w, b = p[name + "/kernel"], p[name + "/bias"]
    k = w.shape[0]
    pt, pb = _same_pads(x.shape[2], k, stride)
    pl, pr = _same_pads(x.shape[3], k, stride)
    xp = F.pad(x, (pl, pr, pt, pb)) if (pt or pb or pl or pr) else x
    return q(F.conv2d(q(xp), qw(w).permute(3, 2, 0, 1), b, stride))


def conv(x, p, name, seperable, stride=1):
    return sepconv(x, p, name, stride) if seperable else dense_conv(x, p, name, stride)


def bn_group(x, p, name, group, stats=None):
    """Training-mode BN over sub-batches of `group` images (one Keras forward per sub-batch)."""
    g, bta = p[name + "/gamma"].view(1, -1, 1, 1), p[name + "/beta"].view(1, -1, 1, 1)
    outs = []
    for s in range(0, x.shape[0], group):
        xs = x[s:s + group]
        m = xs.mean(dim=(0, 2, 3), keepdim=True)
        v = ((xs - m) ** 2).mean(dim=(0, 2, 3), keepdim=True)
        if stats is not None:
            n = xs.shape[0] * xs.shape[2] * xs.shape[3]
            stats.append((name, m.detach().flatten(), (v.detach() * n / max(n - 1, 1)).flatten()))
        outs.append((xs - m) / torch.sqrt(v + BN_EPS) * g + bta)
    return q(torch.cat(outs, 0))


def cnn_block(x, p, blk, group, n_repeats=2, stats=None, seperable=True, batch_norm=True, norm_order="norm_first"):
    """tf_centernet_hourglass.py:87-156 with its options: norm_first (BN on the repeat input, which
    is then the residual's addend) or norm_last (BN on the 2nf-channel output before the ReLU);
    batch_norm=False drops the BN; seperable=False uses Conv2D."""
    t = x
    res = None
    for r in range(n_repeats):
        bn = "%s_bn_%d" % (blk, r)
        if norm_order == "norm_first" and batch_norm:
            t = bn_group(t, p, bn, group, stats)
        y = conv(t, p, "%s_bot_%d" % (blk, r), seperable)
        y = conv(y, p, "%s_cnn_%d" % (blk, r), seperable)
        y = conv(y, p, "%s_out_%d" % (blk, r), seperable)
        if norm_order == "norm_last" and batch_norm:
            y = bn_group(y, p, bn, group, stats)
        y = torch.relu(y)
        res = y if r == 0 else q(y + t)
        t = res
    return res


def pool(x):
    return F.max_pool2d(x, 2, 2, ceil_mode=True)


def up(x):
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def forward(x_nhwc, p, num_classes, group, n_stacks=1, stats=None, seperable=True, batch_norm=True,
            norm_order="norm_first"):
    """x [B,H,W,3] fp32 -> [B,H/4,W/4,4+C] (reg | cls + b_focal)."""
    x = x_nhwc.permute(0, 3, 1, 2)
    v = {"blk0": conv(x, p, "cnn_block_0", seperable, stride=2)}
    blk = dict((b[0], b) for b in blocks(n_stacks))

    def run(name):
        _, i, o = blk[name]
        v[o] = cnn_block(v[i], p, name, group, stats=stats, seperable=seperable, batch_norm=batch_norm,
                         norm_order=norm_order)
        return v[o]
    run("cnn_block_1")
    v["stack_in"] = pool(v["cnn1"])
    for s in range(n_stacks):
        st = "stack_%d_" % (s + 1)
        v["e1"] = pool(q(v["stack_in"] + run(st + "enc_block_1")))
        v["e2"] = pool(q(v["e1"] + run(st + "enc_block_2")))
        v["e3"] = pool(q(v["e2"] + run(st + "enc_block_3")))
        run(st + "enc_block_4a")
        run(st + "enc_block_4b")
        v["e4"] = pool(q(v["e3"] + run(st + "enc_block_4")))
        v["d1res"] = q(run(st + "dec_block_1") + up(v["e4"]))
        run(st + "dec_out_1")
        v["d2res"] = q(run(st + "dec_block_2") + up(v["o1"]))
        run(st + "dec_out_2")
        v["d3res"] = q(run(st + "dec_block_3") + up(v["o2"]))
        run(st + "dec_out_3")
        v["d4res"] = q(run(st + "dec_block_4") + up(v["o3"]))
        run(st + "dec_out_4")
        v["stack_in"] = v["o4"]
    h = v["o4"]
    w = p["cnn_out/kernel"]
    o = F.conv2d(F.pad(q(h), (1, 1, 1, 1)), qw(w).permute(3, 2, 0, 1), p["cnn_out/bias"])
    o = o.permute(0, 2, 3, 1)
    out = torch.cat([o[..., :4], o[..., 4:] + p["b_focal"].view(1, 1, 1, 1)], -1)
    return qg(out)


def model_loss(y_true, y_pred):
    """tf_centernet_hourglass.py:492-505 -> (cls, reg) sums (torch, autograd)."""
    mask = (y_true[..., 4:].max(-1).values > 0).to(y_pred.dtype)
    cls = focal(y_true[..., 4:], y_pred[..., 4:])
    d = y_true[..., :4] - y_pred[..., :4]
    reg = (torch.where(d.abs() < 1, 0.5 * d * d, d.abs()) * mask.unsqueeze(-1)).sum()
    return cls, reg


def loss_and_grads(params, x, targets, num_classes, sub_batch, cls_lambda=2.5, reg_lambda=1.0, **build):
    """Per sub-batch forward + loss; returns (cls_sum, reg_sum, summed grads dict, output).
    build: forward()'s build_model options (n_stacks, seperable, batch_norm, norm_order)."""
    p = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    B = x.shape[0]
    out = forward(x, p, num_classes, sub_batch, **build)
    total_cls = total_reg = 0.0
    tot = 0.0
    for s in range(0, B, sub_batch):
        c, r = model_loss(targets[s:s + sub_batch], out[s:s + sub_batch])
        tot = tot + cls_lambda * c + reg_lambda * r
        total_cls += float(c)
        total_reg += float(r)
    grads = torch.autograd.grad(tot, list(p.values()), allow_unused=True)
    g = {k: (gg if gg is not None else torch.zeros_like(p[k])) for k, gg in zip(p.keys(), grads)}
    return total_cls, total_reg, g, out.detach()


def adam_step(params, grads, m, v, it, lr, B, clip=1.0, b1=0.9, b2=0.999, eps=1e-7):
    """divide_no_nan(g, B), clip_by_global_norm, Keras Adam (t = it + 1); updates in place."""
    gs = {k: g / B for k, g in grads.items()}
    norm = math.sqrt(sum(float((g.double() ** 2).sum()) for g in gs.values()))
    sc = clip / max(norm, clip)
    t = it + 1
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    for k in params:
        g = gs[k] * sc
        m[k] += (g - m[k]) * (1 - b1)
        v[k] += (g * g - v[k]) * (1 - b2)
        params[k] -= lr_t * m[k] / (torch.sqrt(v[k]) + eps)
    return norm


def train_step_reference(params, m, v, it, images, targets, num_classes, sub_batch, lr=1e-3, clip=1.0, **build):
    """One reference train_step on CPU (in place).  Returns (avg_cls, avg_reg)."""
    B = images.shape[0]
    c, r, g, _ = loss_and_grads(params, images, targets, num_classes, sub_batch, **build)
    with torch.no_grad():
        adam_step(params, g, m, v, it, lr, B, clip)
    return c / B, r / B
