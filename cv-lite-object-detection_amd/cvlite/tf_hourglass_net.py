"""Drop-in mirror of CenterNet/tf_hourglass_net.py (the CenterNet trained by train_hourglass_voc.py)
on MI355X.

  build_model(n_filters, n_classes, tmp_pi, n_repeats, n_features, seperable, batch_norm,
              norm_order)                                        :115-394 -> HourglassV2Model
  sigmoid_loss / focal_loss / model_loss(bboxes, masks, outputs, ...)  :396-413
      -> cvl_hourglass_v2_loss (fused, differentiable w.r.t. nothing: a loss read-out; training
         goes through train_step)
  train_step(voc_model, sub_batch_sz, images, bboxes, masks, optimizer, learning_rate, grad_clip,
             cls_lambda, reg_lambda, loss_type)                  :415-447
      -> cvlite.train_hourglass_v2.HourglassV2Trainer (one captured step per (batch, size))
  decode_detections(output, thresh, img_rows, img_cols, img_scale, img_shape)
      the numeric part of obj_detect_results (:451-548): cvl_centernet_scale_decode (box_mode 2)
The plotting of obj_detect_results and show_object_boxes / _parse_image / bbox_flip90 (file IO)
are outside this tier.
"""
import torch

from . import ops_targets as ot
from .centernet_hourglass import scale_decode
from .hourglass_v2_net import HourglassV2Net
from .train_centernet import Adam
from .train_hourglass_v2 import HourglassV2Trainer


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


class HourglassV2Model(object):
    """What build_model returns: model(x, training) -> [B, H/8, W/8, 4, 5+C] fp32 (sigmoid box
    channels, class logits + b_focal), Keras-named parameters in `.net.store`."""

    def __init__(self, net):
        self.net = net
        self._trainers = {}

    def __call__(self, x, training=False, group=None):
        return self.net(x, training=training, group=group)

    @property
    def trainable_variables(self):
        st = self.net.store
        return [st.p(k) for k in st.offsets]


def box_scales(img_rows=448, img_cols=448, img_scale=None):
    """The four per-scale box scales of obj_detect_results (:457-465, :517-524)."""
    if img_scale is None:
        img_scale = [64, 128, 256, max(img_rows, img_cols) if max(img_rows, img_cols) < 512 else 512]
    elif len(img_scale) != 4:
        raise ValueError("img_scale must be size 4.")
    out = list(img_scale[:3])
    out.append(max(img_rows, img_cols) if max(img_rows, img_cols) <= img_scale[3] else img_scale[3])
    return out


def decode_detections(output, thresh=0.50, img_rows=448, img_cols=448, img_scale=None, img_shape=None):
    """obj_detect_results (:451-548, transpose=False) without the plotting: output = one image of the
    model output [S, S, 4, 5 + C] (device or host) -> float64 rows [n, 6] = (x_lower, y_lower,
    box_width, box_height, int(100 p), class index) of every drawn rectangle, in the reference's
    (scale, np.nonzero) order (x = the row axis, as the reference names it; the rectangle is drawn at
    (y_lower, x_lower)).  Classes: the channels after the first when the model has more than one
    class channel (cls_probs[..., 1:]), else channel 0.  img_shape = the source image's (shape[0],
    shape[1]) (default (img_rows, img_cols))."""
    o = torch.as_tensor(output, dtype=torch.float32)
    ns, ch = int(o.shape[2]), int(o.shape[3])
    assert ns == 4, "the v2 decode reads four scales"
    ncls = ch - 4
    cls0, C = (5, ncls - 1) if ncls > 1 else (4, 1)
    return scale_decode(o, ns, ch, cls0, C, 2, box_scales(img_rows, img_cols, img_scale), 8, thresh, img_rows,
                        img_cols, img_shape)


def build_model(n_filters, n_classes, tmp_pi=0.99, n_repeats=2, n_features=256, seperable=True, batch_norm=True,
                norm_order="norm_first", seed=0):
    """tf_hourglass_net.py:115-394, every build option (Conv2D for seperable=False, no BN,
    norm_last)."""
    if norm_order not in ("norm_first", "norm_last"):
        raise ValueError("norm_order must be 'norm_first' or 'norm_last'")
    return HourglassV2Model(HourglassV2Net(n_classes, n_filters=n_filters, tmp_pi=tmp_pi, n_repeats=n_repeats,
                                           n_features=n_features, device=_dev(), seed=seed, seperable=seperable,
                                           batch_norm=batch_norm, norm_order=norm_order))


def model_loss(bboxes, masks, outputs, img_size=448, reg_lambda=0.10, loss_type="sigmoid", eps=1.0e-6):
    """:398-413 -> (total_cls_loss, total_reg_loss) summed over the batch.  outputs: the model's
    [B,S,S,4,5+C] output; masks must be bboxes[..., 4] (what train_hourglass_voc passes: the box
    weight is read from the targets); img_size / reg_lambda / eps are unused, as in the reference."""
    t = torch.as_tensor(bboxes, dtype=torch.float32, device=_dev()).contiguous()
    o = torch.as_tensor(outputs, dtype=torch.float32, device=_dev()).contiguous()
    B, S0, S1, A, R = t.shape
    assert A == 4 and tuple(o.shape) == tuple(t.shape)
    losses, _ = ot.hourglass_v2_loss(o.view(B, S0 * S1, A * R), t.view(B, S0 * S1, A, R), R - 5, loss_type,
                                     reg_is_prob=True)
    s = losses.double().sum(0)
    return float(s[0]), float(s[1])


def train_step(voc_model, sub_batch_sz, images, bboxes, masks, optimizer, learning_rate=1.0e-3, grad_clip=1.0,
               cls_lambda=2.5, reg_lambda=1.0, loss_type="focal"):
    """:415-447 -> (avg_cls_loss, avg_reg_loss).  optimizer: cvlite.train_centernet.Adam (the
    tf.keras.optimizers.Adam() stand-in); masks must be bboxes[..., 4]."""
    images = torch.as_tensor(images, dtype=torch.float32, device=_dev())
    bboxes = torch.as_tensor(bboxes, dtype=torch.float32, device=_dev())
    B, H = int(images.shape[0]), int(images.shape[1])
    key = (B, H, int(sub_batch_sz), float(cls_lambda), float(reg_lambda), loss_type, float(grad_clip))
    tr = voc_model._trainers.get(key)
    if tr is None:
        opt = optimizer if optimizer is not None else Adam()
        tr = voc_model._trainers[key] = HourglassV2Trainer(voc_model.net, B, H, sub_batch_sz, optimizer=opt,
                                                           cls_lambda=cls_lambda, reg_lambda=reg_lambda,
                                                           grad_clip=grad_clip, loss_type=loss_type)
    tr.load_targets(images, bboxes)
    tr.set_lr(learning_rate)
    s = tr.step().double().sum(0).cpu()
    return float(s[0]) / B, float(s[1]) / B
