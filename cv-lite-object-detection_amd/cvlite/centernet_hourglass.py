"""Drop-in mirror of CenterNet/tf_centernet_hourglass.py on MI355X: `build_model` (the separable
hourglass, cvlite.hourglass_net), `train_step` (cvlite.train_centernet: sub-batch BN, fused loss,
clip + Adam, HIP graphs), `format_data` (cvl_centernet_assign), `model_loss` (cvl_det_loss), `nms`
(cvl_nms), `prediction_to_corners` (cvl_fcos_decode: same formula, :355-377)."""
import numpy as np
import torch

from . import _lib
from . import ops_targets as ot
from .fcos import prediction_to_corners  # noqa: F401  (identical formula)


def format_data(gt_labels, img_dim, num_classes, img_pad=None, stride=8):
    """tf_centernet_hourglass.py:379-456 -> (float32 [pad_w/s, pad_h/s, 4+C], num_targets)."""
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, np.float32)]
    gt = np.asarray(gt_labels, dtype=np.float32).reshape(-1, 5)
    n = len(gt)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = gt
    _lib.require_cuda()
    out = ot.centernet_assign(torch.tensor(boxes, device="cuda"), torch.tensor([n], dtype=torch.int32, device="cuda"),
                              torch.tensor(np.asarray(img_dim, np.float32).reshape(1, 2), device="cuda"),
                              (int(img_pad[0]), int(img_pad[1])), num_classes, stride=stride)
    return out[0].cpu().numpy(), n


def model_loss(y_true, y_pred):
    """tf_centernet_hourglass.py:492-505: (cls, reg) summed over the batch."""
    _lib.require_cuda()
    yt = torch.as_tensor(np.asarray(y_true, np.float32) if not torch.is_tensor(y_true) else y_true,
                         dtype=torch.float32).cuda()
    yp = torch.as_tensor(np.asarray(y_pred, np.float32) if not torch.is_tensor(y_pred) else y_pred,
                         dtype=torch.float32).cuda()
    C = yt.shape[-1] - 4
    t = yt.reshape(1, -1, 4 + C).contiguous()
    p = yp.reshape(1, -1, 4 + C)
    losses, _, _ = ot.det_loss(p[..., :4].contiguous(), p[..., 4:].contiguous(), t, C, with_grad=False)
    return losses[0, 0], losses[0, 1]


def nms(bboxes, iou_threshold, sigma=0.3, method="nms"):
    """tf_centernet_hourglass.py:44-85: rows (xmin, ymin, w, h, score, cls) -> list of emitted rows
    (x1, y1, x2, y2, score, cls), classes in python-set order.  method 'nms' (cvl_nms: greedy, IoU >
    iou_threshold suppressed) or 'soft-nms' (cvl_soft_nms: Gaussian decay exp(-iou^2 / sigma); the
    emitted rows carry their decayed scores)."""
    assert method in ["nms", "soft-nms"]
    b = np.array(bboxes, dtype=np.float64)
    classes = list(set(b[:, 5]))
    b[:, 2] = b[:, 0] + b[:, 2]
    b[:, 3] = b[:, 1] + b[:, 3]
    _lib.require_cuda()
    if method == "soft-nms":
        kept = ot.soft_nms(torch.tensor(b, device="cuda"), classes, sigma)
    else:
        kept = ot.nms(torch.tensor(b, device="cuda"), classes, iou_threshold)
    return [row for row in kept.cpu().numpy()]


def build_model(n_classes, tmp_pi=0.99, n_filters=128, n_stacks=1, n_repeats=2, seperable=True, batch_norm=True,
                norm_order="norm_first"):
    """tf_centernet_hourglass.py:163-353 -> cvlite HourglassNet (callable: model(x) -> [B,H/4,W/4,4+C]),
    every build option of the reference: stacked hourglasses, Conv2D instead of SeparableConv2D,
    no BatchNormalization, norm_last."""
    from .hourglass_net import HourglassNet
    if norm_order not in ("norm_first", "norm_last"):
        raise ValueError("norm_order must be 'norm_first' or 'norm_last'")
    _lib.require_cuda()
    return HourglassNet(n_classes, tmp_pi=tmp_pi, n_filters=n_filters, n_stacks=n_stacks, n_repeats=n_repeats,
                        seperable=seperable, batch_norm=batch_norm, norm_order=norm_order)


def train_step(voc_model, sub_batch_sz, images, bboxes, optimizer, cls_lambda=2.5, reg_lambda=1.0,
               learning_rate=1.0e-3, grad_clip=1.0):
    """tf_centernet_hourglass.py:507-564.  images [B,H,W,3] fp32, bboxes = formatted targets
    [B,H/4,W/4,4+C]; optimizer = cvlite.train_centernet.Adam (tf.keras.optimizers.Adam stand-in).
    Returns (avg_cls_loss, avg_reg_loss) = per-batch sums / batch_size."""
    from .train_centernet import CenterNetTrainer
    _lib.require_cuda()
    images = torch.as_tensor(images, dtype=torch.float32).cuda()
    bboxes = torch.as_tensor(bboxes, dtype=torch.float32).cuda()
    B, H, W, _ = images.shape
    key = (B, H, W, int(sub_batch_sz), id(optimizer), float(cls_lambda), float(reg_lambda), float(grad_clip))
    tr = getattr(voc_model, "_trainers", {}).get(key)
    if tr is None:
        tr = CenterNetTrainer(voc_model, B, (H, W), sub_batch_sz=sub_batch_sz, optimizer=optimizer,
                              cls_lambda=cls_lambda, reg_lambda=reg_lambda, grad_clip=grad_clip)
        voc_model._trainers = getattr(voc_model, "_trainers", {})
        voc_model._trainers[key] = tr
    tr.opt.lr_dev.fill_(float(learning_rate))                    # optimizer.lr.assign(learning_rate)
    tr.load_targets(images, bboxes)
    losses = tr.step().double().sum(0).cpu().numpy()
    return float(losses[0]) / B, float(losses[1]) / B


def decode_detections(pred, thresh=0.50, downsample=8, iou_thresh=0.213, img_rows=448, img_cols=448,
                      img_shape=None):
    """The numeric part of obj_detect_results (tf_centernet_hourglass.py:576-656) for one image:
    pred [H,W,4+C] (the model output, device or host) -> (bboxes_raw [n,6] = (x, y, w, h, score%,
    cls), bboxes_nms [m,6] corner rows) via cvl_centernet_decode + cvl_nms.  img_shape = the
    source image's (shape[0], shape[1]) (defaults to (img_rows, img_cols)).  Plotting is outside
    this path."""
    _lib.require_cuda()
    p = torch.as_tensor(pred, dtype=torch.float32).cuda().contiguous()
    H, W, ld = int(p.shape[0]), int(p.shape[1]), int(p.shape[2])
    img_w, img_h = (img_rows, img_cols) if img_shape is None else (img_shape[0], img_shape[1])
    rows = torch.empty((H * W, 6), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.call("cvl_centernet_decode", _lib.ptr(p), ld, H, W, ld - 4, float(downsample), float(thresh),
              float(img_w / img_rows), float(img_h / img_cols), float(img_w), float(img_h), _lib.ptr(rows),
              _lib.ptr(cnt), _lib.stream())
    n = int(cnt.item())
    raw = rows[:n].cpu().numpy()
    if n == 0:
        return raw, np.zeros((0, 6))
    return raw, np.array(nms(raw.copy(), iou_thresh), np.float64).reshape(-1, 6)


def scale_decode(pred, n_scales, ch_per_scale, cls0, num_classes, box_mode, box_scales, stride, thresh, img_rows,
                 img_cols, img_shape=None):
    """cvl_centernet_scale_decode: one image's per-scale decode of the variant CenterNets
    (box_mode 1: tf_centernet_resnet_s8, 2: tf_hourglass_net) -> float64 rows [n, 6] (host)."""
    _lib.require_cuda()
    p = torch.as_tensor(pred, dtype=torch.float32).cuda().contiguous()
    H, W = int(p.shape[0]), int(p.shape[1])
    ld = int(p[0, 0].numel())
    img_w, img_h = (img_rows, img_cols) if img_shape is None else (img_shape[0], img_shape[1])
    rows = torch.empty((n_scales * H * W, 6), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    sc = (_lib.ctypes.c_double * n_scales)(*[float(v) for v in box_scales])
    _lib.call("cvl_centernet_scale_decode", _lib.ptr(p), ld, H, W, int(n_scales), int(ch_per_scale), int(cls0),
              int(num_classes), int(box_mode), sc, float(stride), float(thresh), float(img_w / img_rows),
              float(img_h / img_cols), float(img_w), float(img_h), _lib.ptr(rows), _lib.ptr(cnt), _lib.stream())
    return rows[:int(cnt.item())].cpu().numpy()


def peak_detections(pred, thresh=0.3, K=100, downsample=8, num_classes=None):
    """CenterNet 3x3 max-pool peak decode (cvl_centernet_peak_decode): pred [B, H, W, 4+C] or
    [H, W, 4+C] model output (device or host) -> one float64 array [n <= K, 6] per image of
    (y_lo, x_lo, y_hi, x_hi, prob, class), probability-descending; corners as
    prediction_to_corners (tf_centernet_hourglass.py:355-377) x downsample.  The standard
    CenterNet decode the BASELINE north_star names; the reference's own obj_detect_results decode
    (threshold + NMS) is decode_detections."""
    _lib.require_cuda()
    p = torch.as_tensor(pred, dtype=torch.float32).cuda().contiguous()
    single = p.dim() == 3
    if single:
        p = p.unsqueeze(0)
    B, H, W, ld = (int(v) for v in p.shape)
    C = ld - 4 if num_classes is None else int(num_classes)
    ws = torch.empty(int(_lib.load().cvl_centernet_peak_decode_workspace_size(B, H, W, C)), dtype=torch.uint8,
                     device="cuda")
    dets = torch.zeros((B, K, 6), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    _lib.call("cvl_centernet_peak_decode", _lib.ptr(p), ld, B, H, W, C, float(downsample), float(thresh), int(K),
              _lib.ptr(dets), _lib.ptr(cnt), _lib.ptr(ws), ws.numel(), _lib.stream())
    d, n = dets.cpu().numpy(), cnt.cpu().tolist()
    out = [d[b, :n[b]] for b in range(B)]
    return out[0] if single else out
