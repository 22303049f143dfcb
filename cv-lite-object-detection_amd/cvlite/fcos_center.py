"""Drop-in mirror of FCOS/fcos_center.py (the centre-sampling FCOS variant trained by
train_fcos_center_voc.py) on MI355X.

  format_data(gt_labels, img_dim, num_classes, img_pad, b_dim, strides, center_only)  :149-317
      -> cvl_fcos_center_assign (one batched launch; `format_data_batched` is the device form)
  build_model / prediction_to_corners / model_loss / focal_loss / smooth_l1_loss / iou_loss
      -> the FCOS network and fused loss (fcos_center.py's model and losses are fcos.py's:
         same towers/heads, focal + smooth-L1/IoU + L1 centerness, :319-399)
"""
import numpy as np
import torch

from . import ops_targets as ot
from .fcos import (DEFAULT_STRIDES, _as_tensor, build_model, focal_loss, iou_loss,  # noqa: F401
                   prediction_to_corners, smooth_l1_loss)
from .fcos import model_loss as _fcos_model_loss


def format_data_batched(boxes, nbox, img_dim, pad_hw, num_classes, b_dim=None, strides=None, center_only=False,
                        out=None, num_targets=None):
    """Device form: boxes [B,Nmax,5], nbox [B], img_dim [B,2] -> targets [B,P,5+C], counts [B,5]."""
    return ot.fcos_center_assign(boxes, nbox, img_dim, pad_hw, num_classes,
                                 strides=tuple(strides or DEFAULT_STRIDES), b_dim=tuple(b_dim or (32, 64, 128, 256)),
                                 center_only=center_only, out=out, num_targets=num_targets)


def format_data(gt_labels, img_dim, num_classes, img_pad=None, b_dim=None, strides=None, center_only=False):
    """fcos_center.py:149-317 -> (list of 5 float32 [S,S,5+C] maps, list of per-level counts)."""
    strides = list(strides or DEFAULT_STRIDES)
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, dtype=np.float32)]
    gt = np.asarray(gt_labels, dtype=np.float32).reshape(-1, 5)
    n = len(gt)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = gt
    dims = np.asarray(img_dim, dtype=np.float32).reshape(1, 2)
    tg, nt = format_data_batched(_as_tensor(boxes), _as_tensor(np.array([n], np.int32), torch.int32),
                                 _as_tensor(dims), (int(img_pad[0]), int(img_pad[1])), num_classes, b_dim,
                                 strides, center_only)
    tg = tg[0].cpu().numpy()
    outs, o = [], 0
    for s in strides:
        h, w = int(img_pad[0] / s), int(img_pad[1] / s)
        outs.append(tg[o:o + h * w].reshape(h, w, 5 + num_classes))
        o += h * w
    return outs, [int(v) for v in nt[0].cpu().numpy()]


def model_loss(y_true, y_pred, reg_type="l1", cen_type="l1"):
    """fcos_center.py:365-399 (no `strides` argument, unlike fcos.model_loss).  cen_type="l1" is
    the trained configuration; the focal centerness branch is not implemented (raises)."""
    if cen_type.lower() != "l1":
        raise NotImplementedError("cen_type='focal' (fcos_center.py:386-389) is not on the trained path")
    return _fcos_model_loss(y_true, y_pred, None, reg_type=reg_type, cen_type=cen_type)
