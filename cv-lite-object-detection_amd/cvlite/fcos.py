"""Drop-in mirror of the reference module FCOS/fcos.py on MI355X.

Same names, argument names, defaults and return structures as the reference:
  build_model(num_classes, backbone_model="resnet50")              fcos.py:6-110
  prediction_to_corners(xy_pred, stride)                           fcos.py:112-134
  format_data(gt_labels, img_dim, num_classes, img_pad, areas, strides)  fcos.py:136-378
  smooth_l1_loss / iou_loss / focal_loss / model_loss              fcos.py:380-496
All numeric work runs in the cvlite HIP kernels (include/cvlite.h); there is no CPU fallback.
Differences, by design: maps come back as float32 (the reference stores float64 maps, but its
loss casts them to float32 first; the float32 values are bit-identical); the model is a cvlite
FCOSNet (NHWC torch tensors on the GPU, explicit fwd/bwd) instead of a tf.keras.Model.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import ops_targets as ot
from .fcos_net import FCOSNet

DEFAULT_STRIDES = (8, 16, 32, 64, 128)


def _dev():
    _lib.require_cuda()
    return torch.device("cuda", torch.cuda.current_device())


def _as_tensor(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        return x.detach().to(_dev(), dtype).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=_dev()).contiguous()


class FCOSModel(object):
    """What build_model returns: model(x, training=True) -> list of 5 [B,S,S,5+C] fp32 tensors
    (channels: t, b, l, r, centerness, C class logits), like the reference's Keras model.
    With autograd enabled and training=True the outputs are differentiable w.r.t.
    `trainable_variables` (one torch_ops.NetFunction node: the explicit backward of the same
    kernels the trainer runs), so `torch.autograd.grad(loss, model.trainable_variables)` plays
    the role of the reference's GradientTape (FCOS/train_fcos.py:152-174)."""

    def __init__(self, num_classes, backbone_model="resnet50", seed=0):
        self.net = FCOSNet(num_classes, backbone_model=backbone_model, device=_dev(), seed=seed)
        self.num_classes = num_classes
        self._vars = None

    def __call__(self, x, training=True):
        x = _as_tensor(x)
        B, H, W, _ = x.shape
        if training and torch.is_grad_enabled():
            from .torch_ops import NetFunction
            reg, cls = NetFunction.apply(self.net, x, *self.trainable_variables)
        else:
            reg, cls = self.net.forward(x, train=training)
        shapes, off, P = self.net.layout(B, H, W)
        outs = []
        for l, (h, w) in enumerate(shapes):
            r = reg[:, off[l]:off[l] + h * w, :5]
            c = cls[:, off[l]:off[l] + h * w, :self.num_classes]
            outs.append(torch.cat([r, c], -1).reshape(B, h, w, 5 + self.num_classes))
        return outs

    @property
    def trainable_variables(self):
        """Views of the flat fp32 parameter buffer, in Keras creation order (requires_grad leaves,
        updated in place by the optimizer kernels)."""
        if self._vars is None:
            st = self.net.store
            self._vars = [st.p(k).requires_grad_(True) for k in st.offsets]
        return self._vars


def build_model(num_classes, backbone_model="resnet50"):
    """fcos.py:6-110 (backbone_model "resnet50" -> ResNet-50, anything else -> MobileNetV2 as the
    reference)."""
    return FCOSModel(num_classes, backbone_model=backbone_model)


def prediction_to_corners(xy_pred, stride):
    """fcos.py:112-134: [S,S,>=4] (t, b, l, r) -> float64 [S,S,4] = stride * (y_lo, x_lo, y_hi, x_hi)."""
    p = _as_tensor(xy_pred)
    S0, S1, ld = int(p.shape[0]), int(p.shape[1]), int(p.shape[-1])
    out = torch.empty((S0, S1, 4), dtype=torch.float64, device=p.device)
    _lib.call("cvl_fcos_decode", _lib.ptr(p), ld, S0, S1, ctypes.c_double(float(stride)), _lib.ptr(out),
              _lib.stream())
    return out.cpu().numpy()


def format_data(gt_labels, img_dim, num_classes, img_pad=None, areas=None, strides=None):
    """fcos.py:136-378 on the device (cvl_fcos_assign).  Returns (list of 5 float32 [S,S,5+C]
    numpy maps, list of per-level target counts)."""
    if strides is None:
        strides = DEFAULT_STRIDES
    if areas is not None:
        # the reference defines b_dim only when areas is None (fcos.py:145-147)
        raise NameError("name 'b_dim' is not defined")
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, dtype=np.float32)]
    gt = np.asarray(gt_labels, dtype=np.float32).reshape(-1, 5)
    n = len(gt)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = gt
    dims = np.asarray(img_dim, dtype=np.float32).reshape(1, 2)
    tg, nt = ot.fcos_assign(_as_tensor(boxes), _as_tensor(np.array([n], np.int32), torch.int32),
                            _as_tensor(dims), (int(img_pad[0]), int(img_pad[1])), num_classes,
                            strides=tuple(strides))
    tg = tg[0].cpu().numpy()
    outs, o = [], 0
    for s in strides:
        h, w = int(img_pad[0] / s), int(img_pad[1] / s)
        outs.append(tg[o:o + h * w].reshape(h, w, 5 + num_classes))
        o += h * w
    return outs, [int(v) for v in nt[0].cpu().numpy()]


def _packed_loss(targets, reg, cls, C, reg_type, **kw):
    losses, _, _ = ot.fcos_loss(reg, cls, targets, C, reg_type=reg_type, with_grad=False, **kw)
    return losses[0]


def _as_pred(y):
    """Predictions keep their autograd graph when they already are fp32 device tensors."""
    if isinstance(y, torch.Tensor) and y.is_cuda and y.dtype == torch.float32:
        return y
    return _as_tensor(y)


def model_loss(y_true, y_pred, strides, reg_type="l1", cen_type="l1", cls_lambda=2.5, reg_lambda=1.0):
    """fcos.py:464-496.  y_true: 5 maps [S,S,5+C]; y_pred: 5 tensors [1,S,S,5+C] (index [0], Q11).
    Returns (cls_loss, reg_loss, cen_loss) as 0-d fp32 device tensors; strides/lambdas unused
    exactly as in the reference.  Differentiable w.r.t. y_pred (torch.ops.cvlite.fcos_loss)."""
    from . import torch_ops  # noqa: F401  (registers torch.ops.cvlite.*)
    t = torch.cat([_as_tensor(y).reshape(-1, y.shape[-1]) for y in y_true], 0)
    p = torch.cat([_as_pred(y)[0].reshape(-1, y.shape[-1]) for y in y_pred], 0)
    C = t.shape[-1] - 5
    reg = torch.nn.functional.pad(p[:, :5], (0, 3))[None].contiguous()
    cls = p[None, :, 5:].contiguous()
    l = torch.ops.cvlite.fcos_loss(reg, cls, t[None].contiguous(), C, 1 if reg_type == "iou" else 0)[0]
    cen = l[2] if cen_type.lower() == "l1" else torch.zeros((), device=p.device)
    return l[0], l[1], cen


def focal_loss(labels, logits, alpha=0.25, gamma=2.0):
    """fcos.py:443-462 (sum over all elements, any alpha / gamma >= 0, soft labels) through the
    fused kernel's class path."""
    x = _as_tensor(logits)
    y = _as_tensor(labels)
    C = int(x.shape[-1])
    N = x.numel() // C
    tg = torch.zeros((1, N, 5 + C), dtype=torch.float32, device=x.device)
    tg[0, :, 5:] = y.reshape(N, C)
    reg = torch.zeros((1, N, 8), dtype=torch.float32, device=x.device)
    return _packed_loss(tg, reg, x.reshape(1, N, C).contiguous(), C, "l1", alpha=float(alpha),
                        gamma=float(gamma))[0]


def _masked_reg_loss(xy_true, xy_pred, mask, reg_type, delta=1.0):
    """sum over cells of mask * (per-cell loss summed over the last axis) (fcos.py:380-441): the
    fused kernel's regression path with the float mask in targets[..., 5] (cvl_fcos_loss_ex flag
    32); smooth-L1 rows of k > 4 values run as ceil(k / 4) 4-wide rows of the same cell mask."""
    t = _as_tensor(xy_true)
    p = _as_tensor(xy_pred)
    k = int(t.shape[-1])
    N = t.numel() // k
    if reg_type == "iou":
        assert k == 4
        groups = 1
    else:
        groups = (k + 3) // 4
    tg = torch.zeros((1, N * groups, 6), dtype=torch.float32, device=t.device)
    reg = torch.zeros((1, N * groups, 8), dtype=torch.float32, device=t.device)
    tt = torch.zeros((N, groups * 4), dtype=torch.float32, device=t.device)
    pp = torch.zeros((N, groups * 4), dtype=torch.float32, device=t.device)
    tt[:, :k] = t.reshape(N, k)
    pp[:, :k] = p.reshape(N, k)
    tg[0, :, :4] = tt.reshape(N * groups, 4)
    reg[0, :, :4] = pp.reshape(N * groups, 4)
    tg[0, :, 4] = 0.5                                   # centerness path: sigmoid(0) == 0.5, no loss
    if np.isscalar(mask) or (isinstance(mask, np.ndarray) and mask.ndim == 0):
        mk = torch.full((N,), float(mask), dtype=torch.float32, device=t.device)
    else:
        mk = _as_tensor(mask).reshape(-1)
        assert mk.numel() == N, "mask must have the shape of xy_true without its last axis"
    tg[0, :, 5] = mk.repeat_interleave(groups)
    cls = torch.full((1, N * groups, 1), -100.0, dtype=torch.float32, device=t.device)
    return _packed_loss(tg, reg, cls, 1, reg_type, delta=float(delta), float_mask=True)[1]


def smooth_l1_loss(xy_true, xy_pred, mask=1.0, delta=1.0):
    """fcos.py:380-391 (discontinuous 'smooth L1', Q8: 0.5 d^2 if |d| < delta else |d|) times the
    (float) cell mask, summed over all elements."""
    return _masked_reg_loss(xy_true, xy_pred, mask, "l1", delta)


def iou_loss(xy_true, xy_pred, mask):
    """fcos.py:393-441."""
    return _masked_reg_loss(xy_true, xy_pred, mask, "iou")
