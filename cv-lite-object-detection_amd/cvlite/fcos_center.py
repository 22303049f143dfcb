"""Drop-in mirror of FCOS/fcos_center.py (the centre-sampling FCOS variant trained by
train_fcos_center_voc.py) on MI355X.

  build_model(num_classes, backbone_model)                                      :6-122
      -> FCOSCenterModel over cvlite.fcos_center_net.FCOSCenterNet: the centerness logit is
         `cen_output_l` on the CLS tower and `reg_output_l` has 4 channels (NOT fcos.py's heads)
  format_data(gt_labels, img_dim, num_classes, img_pad, b_dim, strides, center_only)  :149-317
      -> cvl_fcos_center_assign (one batched launch; `format_data_batched` is the device form)
  model_loss(y_true, y_pred, reg_type, cen_type)                                 :365-399
      -> the fused loss (cvl_fcos_loss) with centerness as smooth-L1 of the sigmoid ("l1") or
         focal ("focal", what train_fcos_center_voc.py:194-195 trains)
  prediction_to_corners / focal_loss / smooth_l1_loss / iou_loss: fcos.py's (identical code)
"""
import numpy as np
import torch

from . import ops_targets as ot
from .fcos import (DEFAULT_STRIDES, _as_pred, _as_tensor, _dev, focal_loss, iou_loss,  # noqa: F401
                   prediction_to_corners, smooth_l1_loss)


class FCOSCenterModel(object):
    """What build_model returns: model(x, training=True) -> 5 tensors [B,S,S,5+C] fp32 in the
    reference's channel order (reg 4, centerness 1, classes C).  Differentiable w.r.t.
    `trainable_variables` like cvlite.fcos.FCOSModel."""

    def __init__(self, num_classes, backbone_model="resnet50", seed=0, v1=False):
        from .fcos_center_net import FCOSCenterNet
        self.net = FCOSCenterNet(num_classes, backbone_model=backbone_model, device=_dev(), seed=seed, v1=v1)
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
        return self.net.outputs_nested(reg, cls, H, W)

    @property
    def trainable_variables(self):
        if self._vars is None:
            st = self.net.store
            self._vars = [st.p(k).requires_grad_(True) for k in st.offsets]
        return self._vars


def build_model(num_classes, backbone_model="resnet50"):
    """fcos_center.py:6-122 (ResNet-50 / ResNet-101 backbones)."""
    return FCOSCenterModel(num_classes, backbone_model=backbone_model)


def format_data_batched(boxes, nbox, img_dim, pad_hw, num_classes, b_dim=None, strides=None, center_only=False,
                        out=None, num_targets=None):
    """Device form: boxes [B,Nmax,5], nbox [B], img_dim [B,2] -> targets [B,P,5+C], counts [B,5]."""
    return ot.fcos_center_assign(boxes, nbox, img_dim, pad_hw, num_classes,
                                 strides=tuple(strides or DEFAULT_STRIDES), b_dim=tuple(b_dim or (32, 64, 128, 256)),
                                 center_only=center_only, out=out, num_targets=num_targets)


def _unbatch(tg, nt, img_pad, strides, num_classes):
    tg = tg[0].cpu().numpy()
    outs, o = [], 0
    for s in strides:
        h, w = int(img_pad[0] / s), int(img_pad[1] / s)
        outs.append(tg[o:o + h * w].reshape(h, w, 5 + num_classes))
        o += h * w
    return outs, [int(v) for v in nt[0].cpu().numpy()]


def _single_boxes(gt_labels):
    gt = np.asarray(gt_labels, dtype=np.float32).reshape(-1, 5)
    n = len(gt)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = gt
    return _as_tensor(boxes), _as_tensor(np.array([n], np.int32), torch.int32)


def format_data(gt_labels, img_dim, num_classes, img_pad=None, b_dim=None, strides=None, center_only=False):
    """fcos_center.py:149-317 -> (list of 5 float32 [S,S,5+C] maps, list of per-level counts)."""
    strides = list(strides or DEFAULT_STRIDES)
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, dtype=np.float32)]
    boxes, nbox = _single_boxes(gt_labels)
    dims = np.asarray(img_dim, dtype=np.float32).reshape(1, 2)
    tg, nt = format_data_batched(boxes, nbox, _as_tensor(dims), (int(img_pad[0]), int(img_pad[1])), num_classes,
                                 b_dim, strides, center_only)
    return _unbatch(tg, nt, img_pad, strides, num_classes)


def centre_model_loss(y_true, y_pred, reg_type="l1", cen_type="l1"):
    """The centre variants' model_loss on nested maps through the fused kernel (differentiable
    w.r.t. y_pred, torch.ops.cvlite.fcos_loss): 5 maps [S,S,5+C] and 5 predictions [1,S,S,5+C]
    (reg 4, centerness 1, classes C; index [0] as the reference)."""
    from . import torch_ops  # noqa: F401  (registers torch.ops.cvlite.*)
    t = torch.cat([_as_tensor(y).reshape(-1, y.shape[-1]) for y in y_true], 0)
    p = torch.cat([_as_pred(y)[0].reshape(-1, y.shape[-1]) for y in y_pred], 0)
    C = t.shape[-1] - 5
    reg = torch.nn.functional.pad(p[:, :5], (0, 3))[None].contiguous()
    cls = p[None, :, 5:].contiguous()
    flags = (1 if reg_type == "iou" else 0) | (4 if cen_type.lower() != "l1" else 0)
    l = torch.ops.cvlite.fcos_loss(reg, cls, t[None].contiguous(), C, flags)[0]
    return l[0], l[1], l[2]


def model_loss(y_true, y_pred, reg_type="l1", cen_type="l1"):
    """fcos_center.py:365-399 (no `strides` argument, unlike fcos.model_loss): (cls, reg, cen)."""
    return centre_model_loss(y_true, y_pred, reg_type=reg_type, cen_type=cen_type)
