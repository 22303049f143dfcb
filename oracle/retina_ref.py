"""Numpy restatement of RetinaNet anchor generation + IoU matching (TEST INFRASTRUCTURE).

Follows /root/reference/RetinaNet/retinanet_module.py:163-365 and RetinaNet/utils.py:42-83.
"""
import numpy as np

f32 = np.float32
STRIDES = (8, 16, 32, 64, 128)


def anchor_dims(anchor_sizes=None, aspect_ratios=None, anchor_scales=None):
    """retinanet_module.py:167-219 -> float32 [5, 9, 2] (h, w); ratio outer, scale inner (Q22).
    sqrt/divide run as fp32 tensor ops in the reference (python float -> fp32 tensor)."""
    sizes = [32.0, 64.0, 128.0, 256.0, 512.0] if anchor_sizes is None else list(anchor_sizes)
    ratios = [0.5, 1.0, 2.0] if aspect_ratios is None else list(aspect_ratios)
    scales = [2 ** x for x in [0, 1 / 3, 2 / 3]] if anchor_scales is None else list(anchor_scales)
    out = []
    for area in sorted(x ** 2 for x in sizes):
        lev = []
        for r in ratios:
            h = np.sqrt(f32(area / r))
            w = f32(f32(area) / h)
            for sc in scales:
                lev.append([f32(f32(sc) * h), f32(f32(sc) * w)])
        out.append(lev)
    return np.array(out, dtype=f32)


def get_anchors(dims, cnn_shape, level):
    """retinanet_module.py:221-246: per anchor [S0,S1,4] = (col, row, h, w) (Q21)."""
    ry = np.arange(cnn_shape[0], dtype=np.float32)
    rx = np.arange(cnn_shape[1], dtype=np.float32)
    gx, gy = np.meshgrid(rx, ry)
    base = np.stack([gx, gy, np.ones_like(gx), np.ones_like(gx)], -1).astype(np.float64)
    return [base * np.array([1, 1, d[0], d[1]], np.float64).reshape(1, 1, 4) for d in dims[level]]


def compute_iou(boxes1, boxes2):
    """RetinaNet/utils.py:42-83, fp32 centre-format IoU."""
    b1 = np.asarray(boxes1).astype(f32)
    b2 = np.asarray(boxes2).astype(f32)
    c1 = np.concatenate([b1[:, :2] - b1[:, 2:] / f32(2), b1[:, :2] + b1[:, 2:] / f32(2)], 1)
    c2 = np.concatenate([b2[:, :2] - b2[:, 2:] / f32(2), b2[:, :2] + b2[:, 2:] / f32(2)], 1)
    lu = np.maximum(c1[:, None, :2], c2[:, :2])
    rd = np.minimum(c1[:, None, 2:], c2[:, 2:])
    it = np.maximum(f32(0), rd - lu)
    inter = it[:, :, 0] * it[:, :, 1]
    a1 = b1[:, 2] * b1[:, 3]
    a2 = b2[:, 2] * b2[:, 3]
    union = np.maximum(a1[:, None] + a2 - inter, f32(1e-8))
    return np.clip(inter / union, f32(0), f32(1))


def format_data(gt_labels, img_dim, dims, n_classes, iou_thresh=0.5, img_pad=None):
    """retinanet_module.py:251-365.  Returns ([5][9] float64 [S,S,4+C], num_targets)."""
    if img_pad is None:
        img_pad = img_dim
    gt = np.asarray(gt_labels, dtype=f32).copy()
    scale = np.array([img_dim[0], img_dim[1], img_dim[0], img_dim[1]], dtype=f32).reshape(1, 4)
    gt[:, :4] = gt[:, :4] * scale                       # :277-278 (on a copy, Q26)
    total = 0
    all_out = []
    for lvl, s in enumerate(STRIDES):
        hm, wm = int(img_pad[0] / s), int(img_pad[1] / s)
        anchors = get_anchors(dims, [hm, wm], lvl)
        lev_out = []
        for a in range(len(dims[lvl])):
            out = np.zeros((hm, wm, n_classes + 4))
            flat = anchors[a].reshape(-1, 4)
            ious = compute_iou(gt[:, :4], flat * np.array([s, s, 1.0, 1.0]))
            for b in range(len(gt)):                   # input order, last writer wins (Q23)
                hit = ious[b] > iou_thresh
                n = int(hit.sum())
                total += n
                if n == 0:
                    continue
                av = flat[hit]
                bv = np.repeat(gt[b:b + 1].astype(f32), n, 0)
                yp = av[:, 0].astype(int)
                xp = av[:, 1].astype(int)
                reg = np.stack([(av[:, 0] * s - bv[:, 0]) / av[:, 2],   # :337-353 (linear, Q24)
                                (av[:, 1] * s - bv[:, 1]) / av[:, 3],
                                bv[:, 2] / av[:, 2], bv[:, 3] / av[:, 3]], 1)
                out[yp, xp, :4] = reg
                out[yp, xp, 4 + int(gt[b, 4])] = 1.0
            lev_out.append(out)
        all_out.append(lev_out)
    return all_out, total


def focal_loss(labels, logits, alpha=0.25, gamma=2.0):
    from .fcos_ref import focal_loss as fl
    return fl(labels, logits, alpha, gamma)


def train_loss_targets(x_pred, x_label):
    """retinanet_module.py:403-426 loss part: sum over 5 levels x 9 anchors (mask = any class > 0)."""
    from .fcos_ref import focal_loss as fl, smooth_l1_loss as sl1
    cls = reg = 0.0
    for l in range(len(x_pred)):
        for a in range(len(x_pred[l])):
            p = np.asarray(x_pred[l][a])[0]
            t = np.asarray(x_label[l][a])
            m = (t[..., 4:].max(-1) > 0).astype(np.float64)
            cls += fl(t[..., 4:], p[..., 4:])
            reg += sl1(t[..., :4], p[..., :4], m)
    return cls, reg


# ----------------------------------------------------------------------------------------------
# inference decode (retinanet_module.py:428-529)
# ----------------------------------------------------------------------------------------------
def prediction_to_corners(xy_pred, anchor_dim, stride):
    """retinanet_module.py:428-451: fp32 grid (index * stride, no +0.5) - t * anchor; size =
    t * anchor; corners (y1, x1, y2, x2) = centre -+ size / 2, all in fp32, stored float64."""
    xy = np.asarray(xy_pred, f32)
    ah, aw = f32(anchor_dim[0]), f32(anchor_dim[1])
    gx, gy = np.meshgrid(np.arange(xy.shape[1], dtype=f32), np.arange(xy.shape[0], dtype=f32))
    xc = gx * f32(stride) - xy[..., 1] * aw
    yc = gy * f32(stride) - xy[..., 0] * ah
    bw = xy[..., 3] * aw
    bh = xy[..., 2] * ah
    out = np.zeros(xy.shape[:2] + (4,))
    out[:, :, 0] = yc - bh / f32(2.0)
    out[:, :, 2] = yc + bh / f32(2.0)
    out[:, :, 1] = xc - bw / f32(2.0)
    out[:, :, 3] = xc + bw / f32(2.0)
    return out


def cpu_nms(dets, base_thr):
    """retinanet_module.py:453-481 in the dets' dtype (fp32 in image_detections).  The reference's
    np.argsort(-scores) is an unstable quicksort; this restatement uses a stable sort (ties are
    kept out of the goldens, as for Q1)."""
    dets = np.asarray(dets)
    dt = dets.dtype.type
    x1, y1, x2, y2, scores = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3], dets[:, 4]
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-scores, kind="stable")
    keep = []
    eps = dt(1e-8)
    while len(order) > 0:
        i = order[0]
        keep.append(i)
        xx1 = np.maximum(x1[i], x1[order[1:]])
        yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]])
        yy2 = np.minimum(y2[i], y2[order[1:]])
        w = np.maximum(dt(0.0), xx2 - xx1)
        h = np.maximum(dt(0.0), yy2 - yy1)
        inter = w * h
        ovr = inter / (areas[i] + areas[order[1:]] - inter + eps)
        inds = np.where(ovr <= dt(base_thr))[0]
        order = order[inds + 1]
    return np.array(keep, dtype=np.int64)


def sigmoid32(x):
    """fp32 sigmoid evaluated in float64 and rounded (TF's fp32 kernel: ulp-level parity unpinned)."""
    return (1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))).astype(f32)


def decode_dets(outputs, dims, strides=STRIDES, cls_thresh=0.05):
    """image_detections (:483-519) before NMS: outputs = nested [5][A] arrays [S0,S1,4+C] (one
    image) -> fp32 [n,6] rows (y1, x1, y2, x2, max prob, first-argmax class) with prob >=
    cls_thresh, in (level, anchor, row-major cell) order."""
    rows = []
    for l, lev in enumerate(outputs):
        for a, o in enumerate(lev):
            o = np.array(o, f32)
            o[..., :4] = prediction_to_corners(o[..., :4], dims[l][a], strides[l])
            o[..., 4:] = sigmoid32(o[..., 4:])
            rows.append(o.reshape(-1, o.shape[-1]))
    t = np.concatenate(rows, 0)
    scores = t[:, 4:].max(1)
    labels = t[:, 4:].argmax(1).astype(f32)
    dets = np.concatenate([t[:, :4], scores[:, None], labels[:, None]], 1).astype(f32)
    return dets[dets[:, 4] >= f32(cls_thresh)]


def image_detections(outputs, dims, strides=STRIDES, iou_thresh=0.5, cls_thresh=0.05):
    """image_detections (:483-529) from the model outputs: decode, threshold, cpu_nms."""
    dets = decode_dets(outputs, dims, strides, cls_thresh)
    keep = cpu_nms(dets, iou_thresh)
    return dets[keep] if len(keep) > 0 else dets
