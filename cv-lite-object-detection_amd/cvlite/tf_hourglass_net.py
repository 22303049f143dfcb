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
obj_detect_results / show_object_boxes / _parse_image / bbox_flip90 (plotting and file IO) are
outside this tier.
"""
import torch

from . import ops_targets as ot
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
