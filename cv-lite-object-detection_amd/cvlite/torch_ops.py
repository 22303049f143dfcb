"""PyTorch custom operators (namespace `cvlite`, torch.library) over the C ABI, with autograd.

SURVEY.md §8b's torch custom-op layer: the kernels behind include/cvlite.h as dispatcher ops that
run on the current HIP stream, so a PyTorch user can call them like built-in ops and take
gradients through them (the reference's `tf.GradientTape` usage, FCOS/train_fcos.py:152-174):

  torch.ops.cvlite.conv2d_nhwc(x, w, b, stride, pad)      Keras Conv2D forward (TF 'same' / valid /
                                                          explicit pad), NHWC bf16, HWIO fp32
                                                          master weights; autograd = the dgrad /
                                                          wgrad / bias-grad kernels
  torch.ops.cvlite.fcos_assign(boxes, nbox, img_dim, pad_h, pad_w, C)   fcos.format_data, batched
  torch.ops.cvlite.fcos_loss(reg, cls, targets, C, reg_type)  fcos.model_loss per image
                                                          [B, 3] = (cls, reg, cen); autograd = the
                                                          fused kernel's gradients scaled by the
                                                          upstream per-image, per-term gradients
  torch.ops.cvlite.retina_assign(...) / centernet_splat(...)  RetinaNet / CenterNet targets
  torch.ops.cvlite.sgd_clip_(w, g, v, lr, momentum, inv_bs, clip)  clip_by_global_norm + Keras
                                                          SGD momentum, in place

`NetFunction` makes a whole cvlite network one autograd node: forward = the network's explicit
forward (training-mode BN), backward = its explicit backward (the same kernels FCOSTrainer runs,
so the parameter gradients are bit-identical to the trainer's gradient buffer); the parameters
are its inputs, so torch.autograd.grad(loss, model.trainable_variables) works.
"""
from typing import List, Optional, Tuple

import torch

from . import ops_nn as nn
from . import ops_targets as ot
from .layers import same_pad

BF16 = torch.bfloat16


def _geometry(H, W, k, stride, pad):
    if pad == "same":
        (Ho, pt), (Wo, pl) = same_pad(H, k, stride), same_pad(W, k, stride)
    elif pad == "valid":
        Ho, Wo, pt, pl = (H - k) // stride + 1, (W - k) // stride + 1, 0, 0
    else:
        p = int(pad)
        Ho, Wo, pt, pl = (H + 2 * p - k) // stride + 1, (W + 2 * p - k) // stride + 1, p, p
    return Ho, Wo, pt, pl


def _pad32(n):
    return max(32, (n + 31) // 32 * 32)


def _packs(w, need_dgrad):
    k, _, cin, cout = (int(s) for s in w.shape)
    npad = _pad32(cout)
    wf = torch.empty((npad, k * k * cin), dtype=BF16, device=w.device)
    wd = torch.empty((_pad32(cin), k * k * npad), dtype=BF16, device=w.device) if need_dgrad else None
    nn.pack_conv_weights(w.contiguous(), k, k, cin, cout, cin, npad, wf, _pad32(cin) if need_dgrad else 0,
                         npad if need_dgrad else 0, wd)
    return wf, wd, npad


# ---- conv2d_nhwc --------------------------------------------------------------------------------
@torch.library.custom_op("cvlite::conv2d_nhwc", mutates_args=(), device_types="cuda")
def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride: int, pad: str) -> torch.Tensor:
    """x [B,H,W,Cin] bf16 (Cin % 32 == 0), w [k,k,Cin,Cout] fp32 HWIO (Cout % 8 == 0), b [Cout] or
    None -> [B,Ho,Wo,Cout] bf16 (fp32 accumulation, one rounding)."""
    B, H, W, cin = (int(s) for s in x.shape)
    k, cout = int(w.shape[0]), int(w.shape[3])
    Ho, Wo, pt, pl = _geometry(H, W, k, stride, pad)
    wf, _, npad = _packs(w, False)
    out = torch.empty((B, Ho, Wo, cout), dtype=BF16, device=x.device)
    d = nn.make_desc(nn.FWD, B, cin, k, k, stride, pt, pl, npad, cout, cout,
                     [nn.seg(Ho, Wo, H, W, wf, None if b is None else b.contiguous())])
    nn.conv_igemm(d, x.contiguous(), out)
    return out


@conv2d_nhwc.register_fake
def _(x, w, b, stride, pad):
    B, H, W, _ = x.shape
    Ho, Wo, _, _ = _geometry(int(H), int(W), int(w.shape[0]), stride, pad)
    return x.new_empty((B, Ho, Wo, w.shape[3]), dtype=BF16)


def _conv_setup(ctx, inputs, output):
    x, w, b, stride, pad = inputs
    ctx.save_for_backward(x, w)
    ctx.has_bias = b is not None
    ctx.stride, ctx.pad = stride, pad


def _conv_backward(ctx, gy):
    x, w = ctx.saved_tensors
    B, H, W, cin = (int(s) for s in x.shape)
    k, cout = int(w.shape[0]), int(w.shape[3])
    Ho, Wo, pt, pl = _geometry(H, W, k, ctx.stride, ctx.pad)
    wf, wd, npad = _packs(w, True)
    g = torch.zeros((B, Ho, Wo, npad), dtype=BF16, device=x.device)
    g[..., :cout] = gy.to(BF16)
    dx = dw = db = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty_like(x)
        d = nn.make_desc(nn.DGRAD, B, npad, k, k, ctx.stride, pt, pl, _pad32(cin), cin, cin,
                         [nn.seg(H, W, Ho, Wo, wd)])
        nn.conv_igemm(d, g, dx)
    if ctx.needs_input_grad[1]:
        dw = torch.zeros((k, k, cin, cout), dtype=torch.float32, device=x.device)
        d = nn.make_desc(nn.FWD, B, cin, k, k, ctx.stride, pt, pl, npad, cout, npad, [nn.seg(Ho, Wo, H, W, wf)])
        nn.conv_wgrad(d, x.contiguous(), g, dw)
    if ctx.has_bias and ctx.needs_input_grad[2]:
        db = torch.zeros((cout,), dtype=torch.float32, device=x.device)
        nn.bias_grad(g, npad, 0, cout, 0, Ho * Wo, Ho * Wo, B, db)
    return dx, dw, db, None, None


conv2d_nhwc.register_autograd(_conv_backward, setup_context=_conv_setup)


# ---- targets ------------------------------------------------------------------------------------
@torch.library.custom_op("cvlite::fcos_assign", mutates_args=(), device_types="cuda")
def fcos_assign(boxes: torch.Tensor, nbox: torch.Tensor, img_dim: torch.Tensor, pad_h: int, pad_w: int,
                num_classes: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """fcos.format_data for a batch: boxes [B,N,5] (yc,xc,h,w,cls), nbox [B] i32, img_dim [B,2]
    -> (targets [B,P,5+C] fp32 level-major, num_targets [B,5] i32)."""
    return ot.fcos_assign(boxes.contiguous(), nbox.contiguous(), img_dim.contiguous(), (pad_h, pad_w), num_classes)


@fcos_assign.register_fake
def _(boxes, nbox, img_dim, pad_h, pad_w, num_classes):
    P = sum(h * w for h, w in ot.fcos_level_shapes(pad_h, pad_w))
    B = boxes.shape[0]
    return boxes.new_empty((B, P, 5 + num_classes)), nbox.new_empty((B, 5))


@torch.library.custom_op("cvlite::retina_assign", mutates_args=(), device_types="cuda")
def retina_assign(boxes: torch.Tensor, nbox: torch.Tensor, img_dim: torch.Tensor, pad: int,
                  anchor_dims: torch.Tensor, num_classes: int, iou_thresh: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """RetinaNet.format_data for a batch -> (targets [B, A*sum S^2, 4+C], num_targets [B])."""
    return ot.retina_assign(boxes.contiguous(), nbox.contiguous(), img_dim.contiguous(), pad, anchor_dims,
                            num_classes, iou_thresh)


@retina_assign.register_fake
def _(boxes, nbox, img_dim, pad, anchor_dims, num_classes, iou_thresh):
    A = anchor_dims.shape[1]
    P = sum(A * (pad // s) ** 2 for s in ot.RETINA_STRIDES)
    return boxes.new_empty((boxes.shape[0], P, 4 + num_classes)), nbox.new_empty((boxes.shape[0],))


@torch.library.custom_op("cvlite::centernet_splat", mutates_args=(), device_types="cuda")
def centernet_splat(boxes: torch.Tensor, nbox: torch.Tensor, img_dim: torch.Tensor, pad_h: int, pad_w: int,
                    num_classes: int, stride: int, sigma: float) -> torch.Tensor:
    """tf_centernet.format_data (heatmap splat) for a batch -> [B, pad_h/s, pad_w/s, 5+C]."""
    return ot.centernet_splat(boxes.contiguous(), nbox.contiguous(), img_dim.contiguous(), (pad_h, pad_w),
                              num_classes, stride, sigma)


@centernet_splat.register_fake
def _(boxes, nbox, img_dim, pad_h, pad_w, num_classes, stride, sigma):
    return boxes.new_empty((boxes.shape[0], pad_h // stride, pad_w // stride, 5 + num_classes))


# ---- fused FCOS loss ------------------------------------------------------------------------------
@torch.library.custom_op("cvlite::fcos_loss", mutates_args=(), device_types="cuda")
def fcos_loss(reg: torch.Tensor, cls: torch.Tensor, targets: torch.Tensor, num_classes: int,
              reg_type: int) -> torch.Tensor:
    """fcos.model_loss per image: reg [B,P,>=5] fp32, cls [B,P,>=C] fp32, targets [B,P,5+C]
    -> [B,3] = (cls, reg, cen) (reg_type: cvl_fcos_loss flags, 0 = smooth-L1, 1 = IoU, +4 focal
    centerness, +8 sigmoid reg)."""
    losses, _, _ = ot.fcos_loss(reg.contiguous(), cls.contiguous(), targets.contiguous(), num_classes,
                                reg_type=int(reg_type), with_grad=False)
    return losses


@fcos_loss.register_fake
def _(reg, cls, targets, num_classes, reg_type):
    return reg.new_empty((reg.shape[0], 3))


def _loss_setup(ctx, inputs, output):
    reg, cls, targets, C, reg_type = inputs
    ctx.save_for_backward(reg, cls, targets)
    ctx.C, ctx.reg_type = C, reg_type


def _loss_backward(ctx, g):
    reg, cls, targets = ctx.saved_tensors
    _, d_reg, d_cls = ot.fcos_loss(reg.contiguous(), cls.contiguous(), targets.contiguous(), ctx.C,
                                   reg_type=int(ctx.reg_type), grad_scale=1.0)
    g = g.to(torch.float32)
    # cls term -> class logits; reg term -> ltrb channels 0..3; centerness term -> channel 4;
    # padding channels get exactly zero
    cscale = torch.zeros((reg.shape[0], 1, cls.shape[2]), dtype=torch.float32, device=reg.device)
    cscale[:, 0, :ctx.C] = g[:, 0:1]
    rscale = torch.zeros((reg.shape[0], 1, reg.shape[2]), dtype=torch.float32, device=reg.device)
    rscale[:, 0, :4] = g[:, 1:2]
    rscale[:, 0, 4] = g[:, 2]
    return d_reg * rscale, d_cls * cscale, None, None, None


fcos_loss.register_autograd(_loss_backward, setup_context=_loss_setup)


# ---- optimizer -----------------------------------------------------------------------------------
@torch.library.custom_op("cvlite::sgd_clip_", mutates_args=("w", "v"), device_types="cuda")
def sgd_clip_(w: torch.Tensor, g: torch.Tensor, v: torch.Tensor, lr: torch.Tensor, momentum: float, inv_bs: float,
              clip: float) -> None:
    """In place: g' = clip_by_global_norm(g * inv_bs, clip); v = momentum*v - lr*g'; w += v."""
    nn.sgd_clip_update(w, g, v, lr, momentum, inv_bs, clip)


# ---- whole-network autograd node ------------------------------------------------------------------
class NetFunction(torch.autograd.Function):
    """outputs = net.forward(x) (training-mode BN); backward = net.backward with the head
    gradients (bf16 [B,P,32-padded] as the fused losses write them), returning the parameter
    gradients from the flat gradient buffer.  Inputs: (net, x, *params) with params the store's
    tensors in store order (so autograd routes gradients to model.trainable_variables)."""

    @staticmethod
    def forward(ctx, net, x, *params):
        reg, cls = net.forward(x, train=True)
        ctx.net = net
        ctx.saved_state = net._saved
        ctx.shapes = (reg.shape, cls.shape)
        return reg, cls

    @staticmethod
    def backward(ctx, g_reg, g_cls):
        net = ctx.net
        B, P = ctx.shapes[0][0], ctx.shapes[0][1]
        d_reg = torch.zeros((B, P, 32), dtype=BF16, device=net.device)
        d_cls = torch.zeros((B, P, net.cls_ld), dtype=BF16, device=net.device)
        if g_reg is not None:
            d_reg[..., :g_reg.shape[2]] = g_reg.to(BF16)
        if g_cls is not None:
            d_cls[..., :g_cls.shape[2]] = g_cls.to(BF16)
        net._saved = ctx.saved_state
        net.backward(d_reg, d_cls)
        st = net.store
        grads = [st.g(name).clone() for name in st.offsets]
        return (None, None) + tuple(grads)


def net_params(net) -> List[torch.Tensor]:
    st = net.store
    return [st.p(name) for name in st.offsets]
