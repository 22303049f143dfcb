"""Drop-in mirror of CenterNet/tf_centernet_resnet_s8.py (the CenterNet of
train_centernet_crowdhuman.py) on MI355X.

  build_model(num_classes, n_scales, backbone_model)         :87-208 -> S8Model (ResNet101 for
      "resnet101"; the reference's if/if/else sends every other name, "resnet50" included, to
      MobileNetV2, cvlite.mobilenet_v2)
  prediction_to_corners(xy_pred, box_scales, stride)          :210-241 -> cvl_fcos_v1_decode per scale
  format_data(gt_labels, box_scales, img_dim, num_classes, img_pad, stride)  :243-330
      -> cvl_centernet_s8_assign (bit-exact, float64 as the reference)
  model_loss(y_true, y_pred)                                   :368-385 (read-out on the model output)
  train_step(model, sub_batch_sz, images, bboxes, optimizer, cls_lambda, reg_lambda, learning_rate,
             grad_clip)                                        :387-444 -> S8Trainer
  decode_detections(output, box_scales, thresh, downsample, iou_thresh, img_rows, img_cols, img_shape)
      the numeric part of obj_detect_results (:446-547): cvl_centernet_scale_decode (box_mode 1) +
      nms (:44-85, cvl_nms)
nms: tf_centernet_hourglass's (identical code, cvlite.centernet_hourglass); the plotting and
_parse_image of obj_detect_results are outside this tier.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import ops_targets as ot
from .centernet_hourglass import nms, scale_decode
from .centernet_s8_net import CenterNetS8Net
from .train_centernet_s8 import S8Trainer


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


class S8Model(object):
    """model(x, training) -> [B, H/8, W/8, n_scales, 4+C] fp32 (sigmoid boxes, class logits)."""

    def __init__(self, net):
        self.net = net
        self._trainers = {}

    def __call__(self, x, training=False):
        x = torch.as_tensor(x, dtype=torch.float32).to(_dev()).contiguous()
        reg, cls = self.net.forward(x, train=training)
        return self.net.outputs(reg, cls, x.shape[1], x.shape[2])

    @property
    def trainable_variables(self):
        st = self.net.store
        return [st.p(k) for k in st.offsets]


def build_model(num_classes, n_scales=5, backbone_model="resnet50", seed=0):
    return S8Model(CenterNetS8Net(num_classes, n_scales=n_scales, backbone_model=backbone_model, device=_dev(),
                                  seed=seed))


def prediction_to_corners(xy_pred, box_scales, stride=8):
    """xy_pred [S0, S1, ns, >=4] -> float64 [S0, S1, ns, 4] (y_low, x_low, y_up, x_up) from fp32 math."""
    p = torch.as_tensor(xy_pred, dtype=torch.float32).to(_dev()).contiguous()
    S0, S1, ns = int(p.shape[0]), int(p.shape[1]), int(p.shape[2])
    ld = ns * int(p.shape[3])
    out = torch.empty((ns, S0, S1, 4), dtype=torch.float64, device=p.device)
    for s in range(ns):
        _lib.call("cvl_fcos_v1_decode", ctypes.c_void_p(p[:, :, s].data_ptr()), ld, S0, S1,
                  ctypes.c_float(float(box_scales[s])), ctypes.c_float(float(stride)), _lib.ptr(out[s]), _lib.stream())
    return out.permute(1, 2, 0, 3).cpu().numpy()


def decode_detections(output, box_scales, thresh=0.50, downsample=8, iou_thresh=0.213, img_rows=448, img_cols=448,
                      img_shape=None):
    """obj_detect_results (:446-547) without the plotting: output = one image of the model output
    [S0, S1, n_scales, 4 + C] (device or host) -> (bboxes_raw [n, 6] = (x_low, y_low, w, h, int(100 p),
    class) in the reference's (scale, np.nonzero) order, bboxes_nms [m, 6] corner rows from `nms`).
    img_shape = the source image's (shape[0], shape[1]) (default (img_rows, img_cols))."""
    o = torch.as_tensor(output, dtype=torch.float32)
    ns, ch = int(o.shape[2]), int(o.shape[3])
    raw = scale_decode(o, ns, ch, 4, ch - 4, 1, list(box_scales)[:ns], downsample, thresh, img_rows, img_cols,
                       img_shape)
    if len(raw) == 0:
        return raw, np.zeros((0, 6))
    return raw, np.array(nms(raw.copy(), iou_thresh, method="nms"), np.float64).reshape(-1, 6)


def format_data(gt_labels, box_scales, img_dim, num_classes, img_pad=None, stride=8):
    """:243-330 -> (float32 [pad_w/stride, pad_h/stride, ns, 4+C], num_targets)."""
    if img_pad is None:
        img_pad = img_dim
    lab = np.asarray(gt_labels, np.float64).reshape(-1, 5).astype(np.float32)
    n = len(lab)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = lab
    dev = _dev()
    out = ot.centernet_s8_assign(torch.from_numpy(boxes).to(dev), torch.tensor([n], dtype=torch.int32, device=dev),
                                 torch.tensor([[float(img_dim[0]), float(img_dim[1])]], dtype=torch.float32, device=dev),
                                 (int(img_pad[0]), int(img_pad[1])), num_classes, box_scales, stride=stride)
    return out[0].cpu().numpy(), n


def model_loss(y_true, y_pred):
    """:368-385 on the model output (sigmoid boxes): (cls, reg) sums.  Runs the fused kernel on the
    box logits recovered from the sigmoid outputs (logit(p)); use the trainer for training."""
    t = torch.as_tensor(y_true, dtype=torch.float32, device=_dev()).contiguous()
    o = torch.as_tensor(y_pred, dtype=torch.float32, device=_dev())
    B, S0, S1, ns, R = t.shape
    C = R - 4
    p = o[..., :4].double().clamp(1e-12, 1 - 1e-12)
    reg = torch.log(p / (1 - p)).float().reshape(B, S0 * S1, ns * 4).contiguous()
    cls = o[..., 4:].reshape(B, S0 * S1, ns * C).contiguous()
    losses, _, _ = ot.centernet_s8_loss(reg, cls, t.view(B, S0 * S1, ns, R), C, ns)
    s = losses.double().sum(0)
    return float(s[0]), float(s[1])


def train_step(model, sub_batch_sz, images, bboxes, optimizer=None, cls_lambda=1.0, reg_lambda=1.0,
               learning_rate=1.0e-3, grad_clip=1.0):
    """:387-444 with pre-formatted targets `bboxes` [B,S,S,ns,4+C]; per-image BN (sub_batch_sz 1, the
    trainer's value; other values are accepted for the loss / gradient sums, which do not depend on
    it, while BN statistics stay per image).  Returns (avg_cls, avg_reg)."""
    images = torch.as_tensor(images, dtype=torch.float32, device=_dev())
    bboxes = torch.as_tensor(bboxes, dtype=torch.float32, device=_dev())
    B, H = int(images.shape[0]), int(images.shape[1])
    key = (B, H, float(cls_lambda), float(reg_lambda), float(grad_clip))
    tr = model._trainers.get(key)
    if tr is None:
        mom = getattr(optimizer, "momentum", 0.9)
        tr = model._trainers[key] = S8Trainer(model.net, B, H, cls_lambda=cls_lambda, reg_lambda=reg_lambda,
                                              grad_clip=grad_clip, momentum=mom)
        tr.skip_assign = True
    tr.images.copy_(images)
    tr.targets.copy_(bboxes)
    tr.set_lr(learning_rate)
    s = tr.step().double().sum(0).cpu()
    return float(s[0]) / B, float(s[1]) / B
