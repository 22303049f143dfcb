"""Drop-in mirror of FCOS/fcos_center_v1.py (the centroid-cell FCOS variant trained by
train_fcos_center_v1_voc.py) on MI355X.

  build_model(num_classes, backbone_model)                                    :6-122
      -> FCOSCenterNet(v1=True): the centre network of fcos_center.py with a sigmoid on the
         regression head (applied inside the fused loss when training, in the outputs here)
  prediction_to_corners(xy_pred, box_sc, stride)                              :124-147
      -> cvl_fcos_v1_decode (centre (cell + offset) * stride, size * box_sc)
  format_data(gt_labels, img_dim, num_classes, img_pad, b_dim, strides, center_only)  :149-281
      -> cvl_fcos_center_v1_assign (centroid cell only: (y_off, x_off, h / box_sc, w / box_sc),
         centre score 1, class bits; `format_data_batched` is the device form)
  model_loss(y_true, y_pred)                                                  :283-317
      -> the fused loss: focal classes + focal centerness + smooth-L1 regression (on the model's
         sigmoid outputs) masked by the class targets
  focal_loss / smooth_l1_loss: fcos.py's (identical code)
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import ops_targets as ot
from .fcos import DEFAULT_STRIDES, _as_tensor, focal_loss, smooth_l1_loss  # noqa: F401
from .fcos_center import FCOSCenterModel, _single_boxes, _unbatch, centre_model_loss


def build_model(num_classes, backbone_model="resnet50"):
    """fcos_center_v1.py:6-122."""
    return FCOSCenterModel(num_classes, backbone_model=backbone_model, v1=True)


def prediction_to_corners(xy_pred, box_sc, stride):
    """fcos_center_v1.py:124-147: [S,S,>=4] (y_off, x_off, h, w) -> float64 [S,S,4] corners."""
    p = _as_tensor(xy_pred)
    S0, S1, ld = int(p.shape[0]), int(p.shape[1]), int(p.shape[-1])
    out = torch.empty((S0, S1, 4), dtype=torch.float64, device=p.device)
    _lib.call("cvl_fcos_v1_decode", _lib.ptr(p), ld, S0, S1, ctypes.c_float(float(box_sc)),
              ctypes.c_float(float(stride)), _lib.ptr(out), _lib.stream())
    return out.cpu().numpy()


def format_data_batched(boxes, nbox, img_dim, pad_hw, num_classes, b_dim=None, strides=None, out=None,
                        num_targets=None):
    """Device form: boxes [B,Nmax,5], nbox [B], img_dim [B,2] -> targets [B,P,5+C], counts [B,5]."""
    return ot.fcos_center_v1_assign(boxes, nbox, img_dim, pad_hw, num_classes,
                                    strides=tuple(strides or DEFAULT_STRIDES),
                                    b_dim=tuple(b_dim or (32, 64, 128, 256)), out=out, num_targets=num_targets)


def format_data(gt_labels, img_dim, num_classes, img_pad=None, b_dim=None, strides=None, center_only=False):
    """fcos_center_v1.py:149-281 -> (list of 5 float32 [S,S,5+C] maps, list of per-level counts);
    `center_only` is accepted and unused, as in the reference."""
    strides = list(strides or DEFAULT_STRIDES)
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, dtype=np.float32)]
    boxes, nbox = _single_boxes(gt_labels)
    dims = np.asarray(img_dim, dtype=np.float32).reshape(1, 2)
    tg, nt = format_data_batched(boxes, nbox, _as_tensor(dims), (int(img_pad[0]), int(img_pad[1])), num_classes,
                                 b_dim, strides)
    return _unbatch(tg, nt, img_pad, strides, num_classes)


def model_loss(y_true, y_pred):
    """fcos_center_v1.py:283-317: (cls, reg, cen) with focal centerness; y_pred are the model's
    outputs (sigmoid already applied to the reg channels)."""
    return centre_model_loss(y_true, y_pred, reg_type="l1", cen_type="focal")
