"""Numpy restatement of the reference FCOS target assignment and losses (TEST INFRASTRUCTURE).

Follows /root/reference/FCOS/fcos.py.  The dtype flow is the one TF2 eager gives the reference
when `img_dim` is the fp32 tensor produced by `data_preprocess.resize_and_pad_image`
(train_fcos.py:131-143): every coordinate/ratio is an fp32 op (no fused multiply-add), the
ltrb targets are fp32 values stored in a float64 map, centerness is float64 arithmetic on them.
"""
import numpy as np

f32 = np.float32
STRIDES = (8, 16, 32, 64, 128)          # fcos.py:142-143
B_DIM = (32, 64, 128, 256)              # fcos.py:145-147


def box_level(hpx, wpx, b_dim=B_DIM):
    """fcos.py:168-179: level from max(h, w) in unpadded pixels, half-open bands."""
    m = max(hpx, wpx)
    if m < b_dim[0]:
        return 0
    for l in range(1, len(b_dim)):
        if b_dim[l - 1] <= m < b_dim[l]:
            return l
    return len(b_dim)


def _wrap(i, n):
    # numpy integer indexing wraps negatives (reference relies on plain python indexing)
    return i + n if i < 0 else i


def format_data(gt_labels, img_dim, num_classes, img_pad=None, strides=STRIDES, b_dim=B_DIM):
    """fcos.py:136-378.  gt_labels: float32 [N,5] (yc, xc, h, w normalised; class).
    Returns (list of float64 [Hp/s, Wp/s, 5+C], list num_targets)."""
    gt = np.asarray(gt_labels, dtype=f32)
    H, W = f32(img_dim[0]), f32(img_dim[1])
    if img_pad is None:
        img_pad = (float(H), float(W))
    hpx = gt[:, 2] * H                                        # fcos.py:152-155 (fp32)
    wpx = gt[:, 3] * W
    levels = [box_level(hpx[i], wpx[i], b_dim) for i in range(len(gt))]
    outs, ntgt = [], []
    for na, s in enumerate(strides):
        Hs, Ws = int(img_pad[0] / s), int(img_pad[1] / s)
        out = np.zeros((Hs, Ws, num_classes + 5))
        idx = [i for i in range(len(gt)) if levels[i] == na]
        if not idx:
            outs.append(out)
            ntgt.append(0)
            continue
        sel = gt[idx]
        if len(sel) > 1:                                      # fcos.py:199-207: ascending area
            area = (sel[:, 2] * H) * (sel[:, 3] * W)
            sel = sel[np.argsort(area, kind="stable")]
        hr, wr = f32(H / f32(s)), f32(W / f32(s))             # fcos.py:162-163
        sf = f32(s)
        for row in sel:
            yc, xc, h, w = row[0], row[1], row[2], row[3]
            c0 = f32(f32(yc - f32(0.5) * h) * H)              # fcos.py:211-215
            c1 = f32(f32(xc - f32(0.5) * w) * W)
            c2 = f32(f32(yc + f32(0.5) * h) * H)
            c3 = f32(f32(xc + f32(0.5) * w) * W)
            t0, t1, t2, t3 = f32(c0 / sf), f32(c1 / sf), f32(c2 / sf), f32(c3 / sf)
            ylo = max(0, int(f32(f32(yc - h / f32(2)) * hr)) + 1)   # fcos.py:217-225 (Q3)
            xlo = max(0, int(f32(f32(xc - w / f32(2)) * wr)) + 1)
            yup = min(int(f32(f32(yc + h / f32(2)) * hr)) + 1, Hs)
            xup = min(int(f32(f32(xc + w / f32(2)) * wr)) + 1, Ws)
            ycen = min(int(0.5 * (ylo + yup)), Hs - 1)       # fcos.py:227-230
            xcen = min(int(0.5 * (xlo + xup)), Ws - 1)
            k = 5 + int(row[4])
            ny, nx = yup - ylo, xup - xlo
            yci, xci = _wrap(ycen, Hs), _wrap(xcen, Ws)
            if ny > 0 and nx > 0:                             # fcos.py:233-283
                gy = (np.arange(ylo, yup, dtype=np.float64) + 0.5).astype(f32)[:, None]
                gx = (np.arange(xlo, xup, dtype=np.float64) + 0.5).astype(f32)[None, :]
                tt = np.maximum(f32(0), gy - t0) * np.ones_like(gx)
                bb = np.maximum(f32(0), t2 - gy) * np.ones_like(gx)
                ll = np.maximum(f32(0), gx - t1) * np.ones_like(gy)
                rr = np.maximum(f32(0), t3 - gx) * np.ones_like(gy)
                reg = out[ylo:yup, xlo:xup]
                reg[..., 0], reg[..., 1], reg[..., 2], reg[..., 3] = tt, bb, ll, rr
                a = reg[..., :4]
                lr = (np.minimum(a[..., 0], a[..., 1]) + 1e-8) / (np.maximum(a[..., 0], a[..., 1]) + 1e-8)
                tb = (np.minimum(a[..., 2], a[..., 3]) + 1e-8) / (np.maximum(a[..., 2], a[..., 3]) + 1e-8)
                reg[..., 4] = np.sqrt(lr * tb)
                out[yci, xci, 4] = 1.0
                reg[..., k] = 1
            elif ny > 0:                                      # fcos.py:284-319
                gy = (np.arange(ylo, yup, dtype=np.float64) + 0.5).astype(f32)
                col = out[ylo:yup, xci]
                col[:, 0] = np.maximum(f32(0), gy - t0)
                col[:, 1] = np.maximum(f32(0), t2 - gy)
                col[:, 2] = max(f32(0), f32(f32(xcen + 0.5) - t1))
                col[:, 3] = max(f32(0), f32(f32(t3 - f32(xcen)) - f32(0.5)))
                lr = (np.minimum(col[:, 0], col[:, 1]) + 1e-8) / (np.maximum(col[:, 0], col[:, 1]) + 1e-8)
                col[:, 4] = np.sqrt(lr * 1.0)
                out[yci, xci, 4] = 1.0
                col[:, k] = 1
            elif nx > 0:                                      # fcos.py:320-355
                gx = (np.arange(xlo, xup, dtype=np.float64) + 0.5).astype(f32)
                rw = out[yci, xlo:xup]
                rw[:, 0] = max(f32(0), f32(f32(ycen + 0.5) - t0))
                rw[:, 1] = max(f32(0), f32(f32(t2 - f32(ycen)) - f32(0.5)))
                rw[:, 2] = np.maximum(f32(0), gx - t1)
                rw[:, 3] = np.maximum(f32(0), t3 - gx)
                tb = (np.minimum(rw[:, 2], rw[:, 3]) + 1e-8) / (np.maximum(rw[:, 2], rw[:, 3]) + 1e-8)
                rw[:, 4] = np.sqrt(1.0 * tb)
                out[yci, xci, 4] = 1.0
                rw[:, k] = 1
            else:                                             # fcos.py:356-374
                cell = out[yci, xci]
                cell[0] = max(f32(0), f32(f32(ycen + 0.5) - t0))
                cell[1] = max(f32(0), f32(f32(t2 - f32(ycen)) - f32(0.5)))
                cell[2] = max(f32(0), f32(f32(xcen + 0.5) - t1))
                cell[3] = max(f32(0), f32(f32(t3 - f32(xcen)) - f32(0.5)))
                cell[4] = 1
                cell[k] = 1
        outs.append(out)
        ntgt.append(len(sel))
    return outs, ntgt


def pack_targets(outs):
    """Level-major packed layout used by the device path: [sum S^2, 5+C] float32."""
    return np.concatenate([o.reshape(-1, o.shape[-1]) for o in outs], 0).astype(f32)


# ---------------------------------------------------------------------------------------------
# losses (float64 restatements; fcos.py:380-496)
# ---------------------------------------------------------------------------------------------
def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def focal_loss(labels, logits, alpha=0.25, gamma=2.0):
    """fcos.py:443-462 (plain sum, Q9)."""
    y = np.asarray(labels, np.float32).astype(np.float64)
    x = np.asarray(logits, np.float32).astype(np.float64)
    L = np.log(1.0 + np.exp(-np.abs(x)))
    p = _sig(x)
    t = (y * alpha * L * (1 - p) ** gamma + p ** gamma * (1 - y) * (1 - alpha) * L
         + (1 - y) * (1 - alpha) * np.maximum(x, 0) * p ** gamma
         - y * alpha * np.minimum(x, 0) * (1 - p) ** gamma)
    return float(t.sum())


def smooth_l1_loss(xy_true, xy_pred, mask=1.0, delta=1.0):
    """fcos.py:380-391: 0.5 d^2 if |d| < delta else |d| (discontinuous, Q8)."""
    d = np.asarray(xy_true, np.float32).astype(np.float64) - np.asarray(xy_pred, np.float32).astype(np.float64)
    v = np.where(np.abs(d) < delta, 0.5 * d * d, np.abs(d))
    m = np.expand_dims(np.asarray(mask, np.float64), -1)
    return float((v * m).sum())


def iou_loss(xy_true, xy_pred, mask):
    """fcos.py:393-441 (grid without +0.5; cancels in the IoU)."""
    t = np.asarray(xy_true, np.float32).astype(np.float64)
    p = np.asarray(xy_pred, np.float32).astype(np.float64)
    th = t[..., 0] + t[..., 1]
    tw = t[..., 2] + t[..., 3]
    ph = p[..., 0] + p[..., 1]
    pw = p[..., 2] + p[..., 3]
    ih = np.maximum(0.0, np.minimum(t[..., 1], p[..., 1]) + np.minimum(t[..., 0], p[..., 0]))
    iw = np.maximum(0.0, np.minimum(t[..., 3], p[..., 3]) + np.minimum(t[..., 2], p[..., 2]))
    inter = ih * iw
    union = th * tw + ph * pw - inter
    iou = inter / (union + 1e-12)
    return float((-np.log(iou + 1e-12) * np.asarray(mask, np.float64)).sum())


def model_loss(y_true, y_pred, strides=STRIDES, reg_type="l1", cen_type="l1"):
    """fcos.py:464-496.  y_true: list of [S,S,5+C]; y_pred: list of [1,S,S,5+C] (uses [0], Q11)."""
    cls = reg = cen = 0.0
    for yt, yp in zip(y_true, y_pred):
        yt = np.asarray(yt)
        yp = np.asarray(yp)[0]
        mask = (yt[..., 5:].max(-1) >= 1).astype(np.float64)
        cls += focal_loss(yt[..., 5:], yp[..., 5:])
        if cen_type.lower() == "l1":
            cen += smooth_l1_loss(yt[..., 4], _sig(yp[..., 4].astype(np.float64)), mask=1.0)
        if reg_type == "iou":
            reg += iou_loss(yt[..., :4], yp[..., :4], mask)
        else:
            reg += smooth_l1_loss(yt[..., :4], yp[..., :4], mask=mask)
    return cls, reg, cen


def prediction_to_corners(xy_pred, stride):
    """fcos.py:112-134: [y_low, x_low, y_upp, x_upp] * stride around cell centres."""
    xy = np.asarray(xy_pred, np.float32)
    gy = (np.arange(xy.shape[0], dtype=np.float32) + f32(0.5))[:, None]
    gx = (np.arange(xy.shape[1], dtype=np.float32) + f32(0.5))[None, :]
    out = np.zeros(xy.shape[:2] + (4,))
    out[..., 0] = gy - xy[..., 0]
    out[..., 2] = gy + xy[..., 1]
    out[..., 1] = gx - xy[..., 2]
    out[..., 3] = gx + xy[..., 3]
    return stride * out


def sigmoid32(x):
    """fp32 sigmoid evaluated in float64 and rounded (TF's fp32 kernel: ulp-level parity unpinned)."""
    return (1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))).astype(f32)


def _iou_gt(bi, bj, thr):
    """TF non_max_suppression_op.cc IOUGreaterThanThreshold (fp32, min/max-normalised corners; a
    non-positive area never suppresses) of one box bi against boxes bj [n,4]."""
    bi = np.asarray(bi, f32)
    bj = np.asarray(bj, f32)
    ymin_i, xmin_i = min(bi[0], bi[2]), min(bi[1], bi[3])
    ymax_i, xmax_i = max(bi[0], bi[2]), max(bi[1], bi[3])
    ymin_j, xmin_j = np.minimum(bj[:, 0], bj[:, 2]), np.minimum(bj[:, 1], bj[:, 3])
    ymax_j, xmax_j = np.maximum(bj[:, 0], bj[:, 2]), np.maximum(bj[:, 1], bj[:, 3])
    area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i)
    area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j)
    iy = np.maximum(np.minimum(ymax_i, ymax_j) - np.maximum(ymin_i, ymin_j), f32(0))
    ix = np.maximum(np.minimum(xmax_i, xmax_j) - np.maximum(xmin_i, xmin_j), f32(0))
    inter = iy * ix
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = inter / (area_i + area_j - inter)
    return (iou > f32(thr)) & (area_i > 0) & (area_j > 0)


def combined_non_max_suppression(boxes, scores, max_output_size_per_class, max_total_size, iou_threshold=0.5,
                                 score_threshold=0.05):
    """tf.image.combined_non_max_suppression for one image with q = 1 shared boxes,
    clip_boxes=False, pad_per_class=False (FCOS/infer_fcos.py:55-58), restated from TF's published
    kernel (TF is not installed: parity unpinned at the reference level).  boxes [N,4], scores
    [N,C] fp32 -> (boxes [T,4], scores [T], classes [T], valid) zero padded to T = max_total_size.
    Equal scores: lower box index first per class, then lower class / earlier selection."""
    boxes = np.asarray(boxes, f32)
    scores = np.asarray(scores, f32)
    N, C = scores.shape
    per = min(max_output_size_per_class, N)
    cand = []
    for c in range(C):
        s = scores[:, c]
        idx = np.nonzero(s > f32(score_threshold))[0]
        order = idx[np.argsort(-s[idx], kind="stable")]
        sel = []
        for i in order:
            if len(sel) >= per:
                break
            if sel and _iou_gt(boxes[i], boxes[np.array(sel)], iou_threshold).any():
                continue
            sel.append(i)
        cand += [(s[i], c, k, i) for k, i in enumerate(sel)]
    cand.sort(key=lambda t: (-float(t[0]), t[1], t[2]))
    T = max_total_size
    ob, os_, oc = np.zeros((T, 4), f32), np.zeros(T, f32), np.zeros(T, f32)
    for r, (s, c, _, i) in enumerate(cand[:T]):
        ob[r], os_[r], oc[r] = boxes[i], s, c
    return ob, os_, oc, min(len(cand), T)


def image_detections(outputs, num_classes, center=False, iou_thresh=0.5, cls_thresh=0.05, max_detections=100,
                     max_total_size=100, strides=STRIDES):
    """FCOS/infer_fcos.py:27-62 from the model outputs (5 arrays [S0,S1,5+C], one image):
    fp32 boxes from prediction_to_corners (float64, stored back into the fp32 output), sigmoid
    scores (times the centerness sigmoid with center=True), combined NMS."""
    rows = []
    for l, o in enumerate(outputs):
        o = np.array(o, f32)
        o[..., :4] = prediction_to_corners(o[..., :4], strides[l])
        rows.append(o.reshape(-1, num_classes + 5))
    t = np.concatenate(rows, 0)
    sc = sigmoid32(t[:, 5:])
    if center:
        sc = sigmoid32(t[:, 4])[:, None] * sc
    return combined_non_max_suppression(t[:, :4], sc, max_detections, max_total_size, iou_thresh, cls_thresh)


def center_format_data(gt_labels, img_dim, num_classes, img_pad=None, b_dim=None, strides=None,
                       center_only=False):
    """FCOS/fcos_center.py:149-317 (numpy >= 2 scalar promotion: python scalars join fp32 as fp32):
    per level, boxes by max(h, w) px against b_dim, ascending area (stable: ties avoided, as Q1),
    3x3 (or centre-only) cells around int(centre * img_dim / stride + 0.5); centerness max of
    1 / 0.5 / 0.25, ltrb from the last box, class bits OR-ed -> (5 float64 maps, counts)."""
    strides = list(STRIDES) if strides is None else list(strides)
    b_dim = [32, 64, 128, 256] if b_dim is None else list(b_dim)
    dim = np.asarray(img_dim, f32)
    pad = dim if img_pad is None else np.asarray(img_pad, f32)
    gt = np.asarray(gt_labels, f32).reshape(-1, 5)
    gh, gw = gt[:, 2] * dim[0], gt[:, 3] * dim[1]
    m = np.maximum(gw, gh)
    outs, counts = [], []
    for na, stride in enumerate(strides):
        hr, wr = dim[0] / f32(stride), dim[1] / f32(stride)
        hmax, wmax = int(pad[0] / f32(stride)), int(pad[1] / f32(stride))
        out = np.zeros((hmax, wmax, num_classes + 5))
        if na == 0:
            idx = np.nonzero(m < b_dim[0])[0]
        elif na == len(strides) - 1:
            idx = np.nonzero(m >= b_dim[-1])[0]
        else:
            idx = np.nonzero((m >= b_dim[na - 1]) & (m < b_dim[na]))[0]
        lab = gt[idx]
        if len(lab) > 1:
            lab = lab[np.argsort(np.multiply(lab[:, 2] * dim[0], lab[:, 3] * dim[1]), kind="stable")]
        offs = [0] if center_only else [-1, 0, 1]
        for t in lab:
            c0 = (t[0] - f32(0.5) * t[2]) * dim[0] / f32(stride)
            c1 = (t[1] - f32(0.5) * t[3]) * dim[1] / f32(stride)
            c2 = (t[0] + f32(0.5) * t[2]) * dim[0] / f32(stride)
            c3 = (t[1] + f32(0.5) * t[3]) * dim[1] / f32(stride)
            yc, xc = int(t[0] * hr + f32(0.5)), int(t[1] * wr + f32(0.5))
            for x in [xc - o for o in offs if xc - o >= 0]:
                for y in [yc - o for o in offs if yc - o >= 0]:
                    if y >= hmax or x >= wmax:
                        continue
                    yo, xo = yc - y, xc - x
                    sc = 1.0 if (yo == 0 and xo == 0) else (0.25 if abs(yo) == 1 and abs(xo) == 1 else 0.5)
                    if sc >= out[y, x, 4]:
                        out[y, x, 4] = sc
                    out[y, x, :4] = [f32(y + 0.5) - c0, (c2 - f32(y)) - f32(0.5),
                                     f32(x + 0.5) - c1, (c3 - f32(x)) - f32(0.5)]
                    out[y, x, 5 + int(t[4])] = 1.0
        outs.append(out)
        counts.append(len(lab))
    return outs, counts


def center_v1_prediction_to_corners(xy_pred, box_sc, stride):
    """FCOS/fcos_center_v1.py:124-147: fp32 tensor math (grid + offset) * stride, size * box_sc,
    centre -+ size / 2, stored into a float64 array."""
    p = np.asarray(xy_pred, np.float32)
    gy, gx = np.meshgrid(np.arange(p.shape[0], dtype=np.float32), np.arange(p.shape[1], dtype=np.float32),
                         indexing="ij")
    f32 = np.float32
    yc = (gy + p[..., 0]) * f32(stride)
    xc = (gx + p[..., 1]) * f32(stride)
    bh = p[..., 2] * f32(box_sc)
    bw = p[..., 3] * f32(box_sc)
    out = np.zeros(p.shape[:2] + (4,))
    out[..., 0], out[..., 2] = yc - bh / f32(2.0), yc + bh / f32(2.0)
    out[..., 1], out[..., 3] = xc - bw / f32(2.0), xc + bw / f32(2.0)
    return out


def center_v1_format_data(gt_labels, img_dim, num_classes, img_pad=None, b_dim=None, strides=None):
    """FCOS/fcos_center_v1.py:149-281 (numpy >= 2 promotion): level by max(h, w) px against b_dim,
    ascending area; each box writes its centroid cell int(centre * img_dim / stride):
    (y_off, x_off, h / box_sc, w / box_sc), centre 1, class bit; box_sc = b_dim[l] or max(img_dim)."""
    strides = list(STRIDES) if strides is None else list(strides)
    b_dim = [32, 64, 128, 256] if b_dim is None else list(b_dim)
    dim = np.asarray(img_dim, f32)
    pad = dim if img_pad is None else np.asarray(img_pad, f32)
    gt = np.asarray(gt_labels, f32).reshape(-1, 5)
    gh, gw = gt[:, 2] * dim[0], gt[:, 3] * dim[1]
    m = np.maximum(gw, gh)
    outs, counts = [], []
    for na, stride in enumerate(strides):
        hmax, wmax = int(pad[0] / f32(stride)), int(pad[1] / f32(stride))
        out = np.zeros((hmax, wmax, num_classes + 5))
        if na == 0:
            sc, idx = f32(b_dim[0]), np.nonzero(m < b_dim[0])[0]
        elif na == len(strides) - 1:
            sc, idx = max(dim[0], dim[1]), np.nonzero(m >= b_dim[-1])[0]
        else:
            sc, idx = f32(b_dim[na]), np.nonzero((m >= b_dim[na - 1]) & (m < b_dim[na]))[0]
        lab = gt[idx]
        if len(lab) > 1:
            lab = lab[np.argsort(np.multiply(lab[:, 2] * dim[0], lab[:, 3] * dim[1]), kind="stable")]
        for t in lab:
            ry, rx = t[0] * dim[0], t[1] * dim[1]
            yc, xc = int(ry / f32(stride)), int(rx / f32(stride))
            out[yc, xc, :4] = [(ry - f32(yc * stride)) / f32(stride), (rx - f32(xc * stride)) / f32(stride),
                               (t[2] * dim[0]) / sc, (t[3] * dim[1]) / sc]
            out[yc, xc, 4] = 1.0
            out[yc, xc, 5 + int(t[4])] = 1.0
        outs.append(out)
        counts.append(len(lab))
    return outs, counts


def center_model_loss(y_true, y_pred, reg_type="l1", cen_type="l1", reg_sigmoid=False):
    """FCOS/fcos_center.py:365-399 (cen_type "l1" | "focal") and, with reg_sigmoid=True and
    cen_type="focal", FCOS/fcos_center_v1.py:283-317 fed the raw head logits (the v1 model applies
    the sigmoid to the reg head, fcos_center_v1.py:115).  y_pred: list of [1,S,S,5+C] raw outputs."""
    cls = reg = cen = 0.0
    for yt, yp in zip(y_true, y_pred):
        yt = np.asarray(yt)
        yp = np.asarray(yp, np.float32)[0].astype(np.float64)
        mask = (yt[..., 5:].max(-1) >= 1).astype(np.float64)
        cls += focal_loss(yt[..., 5:], yp[..., 5:])
        if cen_type.lower() == "l1":
            cen += smooth_l1_loss(yt[..., 4], _sig(yp[..., 4]), mask=1.0)
        else:
            cen += focal_loss(yt[..., 4], yp[..., 4])
        r = _sig(yp[..., :4]) if reg_sigmoid else yp[..., :4]
        if reg_type == "iou":
            reg += iou_loss(yt[..., :4], r, mask)
        else:
            reg += smooth_l1_loss(yt[..., :4], r, mask=mask)
    return cls, reg, cen
