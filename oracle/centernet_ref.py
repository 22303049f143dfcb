"""Numpy restatement of the CenterNet targets, splat, loss and decode (TEST INFRASTRUCTURE).

Follows /root/reference/CenterNet/tf_centernet_hourglass.py (format_data :379-456, model_loss
:492-505, nms :44-85, bboxes_iou :22-42) and CenterNet/tf_centernet.py (center_dist_1d/2d :6-19,
format_data :152-342).  fp32 coordinate math as TF2 eager gives it with an fp32 `img_dim` tensor.
"""
import numpy as np

from .fcos_ref import focal_loss, smooth_l1_loss

f32 = np.float32


def _sorted_by_area(gt, H, W):
    if len(gt) <= 1:
        return gt
    area = (gt[:, 2] * H) * (gt[:, 3] * W)
    return gt[np.argsort(area, kind="stable")]


def _coords(row, H, W):
    yc, xc, h, w = row[0], row[1], row[2], row[3]
    return (f32(f32(yc - f32(0.5) * h) * H), f32(f32(xc - f32(0.5) * w) * W),
            f32(f32(yc + f32(0.5) * h) * H), f32(f32(xc + f32(0.5) * w) * W))


def hourglass_format_data(gt_labels, img_dim, num_classes, img_pad=None, stride=8):
    """tf_centernet_hourglass.py:379-456: hard one-hot at the centroid cell (Q30)."""
    gt = np.asarray(gt_labels, dtype=f32)
    H, W = f32(img_dim[0]), f32(img_dim[1])
    if img_pad is None:
        img_pad = (float(H), float(W))
    hm, wm = int(img_pad[1] / stride), int(img_pad[0] / stride)   # swapped, harmless if square
    pad_y = int(f32(f32(f32(img_pad[1]) - W) / f32(2.0)))
    pad_x = int(f32(f32(f32(img_pad[0]) - H) / f32(2.0)))
    out = np.zeros((hm, wm, num_classes + 4))
    if len(gt) == 0:
        return out, 0
    sf = f32(stride)
    for row in _sorted_by_area(gt, H, W):
        c0, c1, c2, c3 = _coords(row, H, W)
        ycf = f32(f32(c0 + c2) / f32(2.0))
        xcf = f32(f32(c1 + c3) / f32(2.0))
        yc = int(f32(f32(f32(pad_y) + ycf) / sf))
        xc = int(f32(f32(f32(pad_x) + xcf) / sf))
        off = [f32(f32(yc + 0.5) - f32(f32(f32(pad_y) + c0) / sf)),
               f32(f32(f32(f32(f32(pad_y) + c2) / sf) - f32(yc)) - f32(0.5)),
               f32(f32(xc + 0.5) - f32(f32(f32(pad_x) + c1) / sf)),
               f32(f32(f32(f32(f32(pad_x) + c3) / sf) - f32(xc)) - f32(0.5))]
        out[yc, xc, :4] = off
        out[yc, xc, 4 + int(row[4])] = 1.0
    return out, len(gt)


def hourglass_model_loss(y_true, y_pred):
    """tf_centernet_hourglass.py:492-505 -> (cls, reg)."""
    y = np.asarray(y_true)
    p = np.asarray(y_pred)
    mask = (y[..., 4:].max(-1) > 0).astype(np.float64)
    return focal_loss(y[..., 4:], p[..., 4:]), smooth_l1_loss(y[..., :4], p[..., :4], mask)


def center_dist_1d(grid_x, mu_x=0.0, spread=2.0):
    """tf_centernet.py:6-10 (inverse power, Q32)."""
    g = 1.0 / np.power(np.asarray(grid_x, np.float64) - mu_x, spread)
    return g / g.max()


def center_dist_2d(grid_x, grid_y, mu_x=0.0, mu_y=0.0, spread=2.0):
    """tf_centernet.py:12-19."""
    gx = 1.0 / np.power(np.asarray(grid_x, np.float64) - mu_x, spread)
    gy = 1.0 / np.power(np.asarray(grid_y, np.float64) - mu_y, spread)
    return gx * gy / (gx * gy).max()


def splat_format_data(gt_labels, img_dim, num_classes, img_pad=None, stride=8, sigma=0.25):
    """tf_centernet.py:152-342: ltrb over the sigma sub-box + inverse-power centre splat in ch4."""
    gt = np.asarray(gt_labels, dtype=f32)
    H, W = f32(img_dim[0]), f32(img_dim[1])
    if img_pad is None:
        img_pad = (float(H), float(W))
    sf = f32(stride)
    hr, wr = f32(H / sf), f32(W / sf)
    Hs, Ws = int(img_pad[0] / stride), int(img_pad[1] / stride)
    ylim, xlim = int(f32(H / sf)), int(f32(W / sf))
    out = np.zeros((Hs, Ws, num_classes + 5))
    spread = 8.0                                                # :206-207 (tmp_std forced to 8)
    sg = f32(sigma)
    for row in _sorted_by_area(gt, H, W):
        c0, c1, c2, c3 = _coords(row, H, W)
        t0, t1, t2, t3 = f32(c0 / sf), f32(c1 / sf), f32(c2 / sf), f32(c3 / sf)
        ycen = int(f32(row[0] * hr))
        xcen = int(f32(row[1] * wr))
        ylo = max(0, 1 + int(f32(f32(row[0] - f32(sg * row[2]) / f32(2)) * hr)))
        xlo = max(0, 1 + int(f32(f32(row[1] - f32(sg * row[3]) / f32(2)) * wr)))
        yup = min(1 + int(f32(f32(row[0] + f32(sg * row[2]) / f32(2)) * hr)), ylim)
        xup = min(1 + int(f32(f32(row[1] + f32(sg * row[3]) / f32(2)) * wr)), xlim)
        k = 5 + int(row[4])
        if yup - ylo > 0 and xup - xlo > 0:
            gyd = np.arange(ylo, yup, dtype=np.float64) + 0.5
            gxd = np.arange(xlo, xup, dtype=np.float64) + 0.5
            gx, gy = np.meshgrid(gxd, gyd)
            gy32, gx32 = gy.astype(f32), gx.astype(f32)
            reg = out[ylo:yup, xlo:xup]
            reg[..., 0] = np.maximum(f32(0), gy32 - t0)
            reg[..., 1] = np.maximum(f32(0), t2 - gy32)
            reg[..., 2] = np.maximum(f32(0), gx32 - t1)
            reg[..., 3] = np.maximum(f32(0), t3 - gx32)
            nx, ny = int(0.5 * (xlo + xup)), int(0.5 * (ylo + yup))
            reg[..., 4] = center_dist_2d(gx, gy, nx, ny, spread)
            out[ny, nx, 4] = 1.0
            reg[..., k] = 1
        elif yup - ylo > 0:
            gyd = np.arange(ylo, yup, dtype=np.float64) + 0.5
            col = out[ylo:yup, xcen]
            col[:, 0] = np.maximum(f32(0), gyd.astype(f32) - t0)
            col[:, 1] = np.maximum(f32(0), t2 - gyd.astype(f32))
            col[:, 2] = max(f32(0), f32(f32(xcen + 0.5) - t1))
            col[:, 3] = max(f32(0), f32(f32(t3 - f32(xcen)) - f32(0.5)))
            ny = int(0.5 * (ylo + yup))
            col[:, 4] = center_dist_1d(gyd, ny, spread)
            out[ny, xcen, 4] = 1.0
            col[:, k] = 1
        elif xup - xlo > 0:
            gxd = np.arange(xlo, xup, dtype=np.float64) + 0.5
            rw = out[ycen, xlo:xup]
            rw[:, 0] = max(f32(0), f32(f32(ycen + 0.5) - t0))
            rw[:, 1] = max(f32(0), f32(f32(t2 - f32(ycen)) - f32(0.5)))
            rw[:, 2] = np.maximum(f32(0), gxd.astype(f32) - t1)
            rw[:, 3] = np.maximum(f32(0), t3 - gxd.astype(f32))
            nx = int(0.5 * (xlo + xup))
            rw[:, 4] = center_dist_1d(gxd, nx, spread)
            out[ycen, nx, 4] = 1.0
            rw[:, k] = 1
        else:
            cell = out[ycen, xcen]
            cell[0] = max(f32(0), f32(f32(ycen + 0.5) - t0))
            cell[1] = max(f32(0), f32(f32(t2 - f32(ycen)) - f32(0.5)))
            cell[2] = max(f32(0), f32(f32(xcen + 0.5) - t1))
            cell[3] = max(f32(0), f32(f32(t3 - f32(xcen)) - f32(0.5)))
            cell[4] = 1
            cell[k] = 1
    return out


def bboxes_iou(b1, b2):
    """tf_centernet_hourglass.py:22-42 (corner format, float64, floor at fp32 eps)."""
    b1 = np.asarray(b1, np.float64)
    b2 = np.asarray(b2, np.float64)
    a1 = (b1[..., 2] - b1[..., 0]) * (b1[..., 3] - b1[..., 1])
    a2 = (b2[..., 2] - b2[..., 0]) * (b2[..., 3] - b2[..., 1])
    lu = np.maximum(b1[..., :2], b2[..., :2])
    rd = np.minimum(b1[..., 2:], b2[..., 2:])
    it = np.maximum(rd - lu, 0.0)
    inter = it[..., 0] * it[..., 1]
    return np.maximum(inter / (a1 + a2 - inter), np.finfo(np.float32).eps)


def nms(bboxes, iou_threshold):
    """tf_centernet_hourglass.py:44-85, method='nms'. Input rows (x, y, w, h, score, cls)."""
    bb = np.array(bboxes, np.float64)
    bb[:, 2] = bb[:, 0] + bb[:, 2]
    bb[:, 3] = bb[:, 1] + bb[:, 3]
    best = []
    for c in list(set(bb[:, 5])):                 # python set order, as the reference
        cb = bb[bb[:, 5] == c]
        while len(cb) > 0:
            i = int(np.argmax(cb[:, 4]))
            b = cb[i]
            best.append(b.copy())
            cb = np.concatenate([cb[:i], cb[i + 1:]])
            iou = bboxes_iou(b[np.newaxis, :4], cb[:, :4])
            keep = ~(iou > iou_threshold)
            cb = cb[keep & (cb[:, 4] > 0)]
    return np.array(best, np.float64).reshape(-1, 6)


def soft_nms(bboxes, sigma=0.3):
    """tf_centernet_hourglass.py:44-85, method='soft-nms' (Gaussian decay, float64).  Input rows
    (x, y, w, h, score, cls); output rows (x1, y1, x2, y2, decayed score, cls) in emission order."""
    bb = np.array(bboxes, np.float64)
    bb[:, 2] = bb[:, 0] + bb[:, 2]
    bb[:, 3] = bb[:, 1] + bb[:, 3]
    best = []
    for c in list(set(bb[:, 5])):
        cb = bb[bb[:, 5] == c]
        while len(cb) > 0:
            i = int(np.argmax(cb[:, 4]))
            b = cb[i]
            best.append(b.copy())
            cb = np.concatenate([cb[:i], cb[i + 1:]])
            iou = bboxes_iou(b[np.newaxis, :4], cb[:, :4])
            cb[:, 4] = cb[:, 4] * np.exp(-(1.0 * iou ** 2 / sigma))
            cb = cb[cb[:, 4] > 0.0]
    return np.array(best, np.float64).reshape(-1, 6)


def prediction_to_corners(xy_pred, stride):
    """tf_centernet_hourglass.py:355-377: fp32 grid (cell + 0.5) -+ ltrb, stored float64, * stride."""
    xy = np.asarray(xy_pred, np.float32)
    H, W = xy.shape[:2]
    ch = np.arange(H, dtype=np.float32) + np.float32(0.5)
    cw = np.arange(W, dtype=np.float32) + np.float32(0.5)
    gx, gy = np.meshgrid(cw, ch)
    out = np.zeros((H, W, 4))
    out[:, :, 0] = gy - xy[..., 0]
    out[:, :, 2] = gy + xy[..., 1]
    out[:, :, 1] = gx - xy[..., 2]
    out[:, :, 3] = gx + xy[..., 3]
    return stride * out


def sigmoid32(x):
    """fp32 sigmoid (tf.nn.sigmoid): evaluated in float64, rounded to fp32 (TF's own fp32 kernel
    is an implementation detail not available here: parity unpinned at the ulp level)."""
    return (1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))).astype(np.float32)


def decode_cells(pred, thresh=0.5, downsample=8, img_rows=448, img_cols=448, img_width=448, img_height=448):
    """The per-cell part of obj_detect_results (tf_centernet_hourglass.py:576-650): rows
    (x_low, y_low, w, h, int(100 p), label) of the cells with max class probability >= thresh, in
    np.nonzero order -> the input of `nms`."""
    pred = np.asarray(pred, np.float32)
    reg = prediction_to_corners(pred[:, :, :4], downsample)
    probs = sigmoid32(pred[:, :, 4:])
    pmax = probs.max(axis=2)
    lab = probs.argmax(axis=2)
    w_ratio = img_width / img_rows
    h_ratio = img_height / img_cols
    rows = []
    xs, ys = np.nonzero(np.where(pmax >= thresh, 1, 0))
    for xc, yc in zip(xs, ys):
        b = reg[xc, yc, :]
        p = int(pmax[xc, yc] * 100)
        x_low, y_low = h_ratio * b[1], w_ratio * b[0]
        x_upp, y_upp = h_ratio * b[3], w_ratio * b[2]
        bw, bh = x_upp - x_low, y_upp - y_low
        if bw > img_width:
            bw = img_width
        if bh > img_height:
            bh = img_height
        if x_low < 0:
            x_low = 0
        if y_low < 0:
            y_low = 0
        rows.append(np.array([x_low, y_low, bw, bh, p, lab[xc, yc]], np.float64))
    return np.array(rows, np.float64).reshape(-1, 6)


def decode_s8_cells(output, box_scales, thresh=0.5, downsample=8, img_rows=448, img_cols=448, img_width=448,
                    img_height=448):
    """The numeric part of tf_centernet_resnet_s8.obj_detect_results (CenterNet/
    tf_centernet_resnet_s8.py:455-547): output [S0, S1, ns, 4 + C] -> the rows (x_low, y_low, w, h,
    int(100 p), label) it hands to `nms`, scale-major, np.nonzero order within a scale.  Corners as
    prediction_to_corners (:210-241): fp32 (grid + offset) * stride and size * box_scale (the scale an
    fp32 operand), corners +- size / 2 in fp32, then float64."""
    o = np.asarray(output, np.float32)
    S0, S1, ns, ch = o.shape
    C = ch - 4
    w_ratio, h_ratio = img_width / img_rows, img_height / img_cols
    gy, gx = np.meshgrid(np.arange(S0, dtype=np.float32), np.arange(S1, dtype=np.float32), indexing="ij")
    rows = []
    for s in range(ns):
        sc = np.float32(box_scales[s])
        st = np.float32(downsample)
        xc = (gx + o[:, :, s, 1]) * st
        yc = (gy + o[:, :, s, 0]) * st
        bw = o[:, :, s, 3] * sc
        bh = o[:, :, s, 2] * sc
        two = np.float32(2.0)
        corners = np.stack([yc - bh / two, xc - bw / two, yc + bh / two, xc + bw / two], -1).astype(np.float64)
        probs = sigmoid32(o[:, :, s, 4:])
        pmax = probs.max(axis=2) if C > 1 else probs[:, :, 0]
        lab = probs.argmax(axis=2) if C > 1 else np.zeros((S0, S1), np.int64)
        xs, ys = np.nonzero(np.where(pmax >= thresh, 1, 0))
        for xi, yi in zip(xs, ys):
            b = corners[xi, yi]
            p = int(pmax[xi, yi] * np.float32(100))
            x_low, y_low = h_ratio * b[1], w_ratio * b[0]
            x_upp, y_upp = h_ratio * b[3], w_ratio * b[2]
            bw_, bh_ = x_upp - x_low, y_upp - y_low
            if bw_ > img_width:
                bw_ = img_width
            if bh_ > img_height:
                bh_ = img_height
            if x_low < 0:
                x_low = 0
            if y_low < 0:
                y_low = 0
            rows.append([x_low, y_low, bw_, bh_, p, lab[xi, yi]])
    return np.array(rows, np.float64).reshape(-1, 6)


def decode_hg2_cells(output, thresh=0.5, img_rows=448, img_cols=448, box_scales=(64, 128, 256, 448), img_width=448,
                     img_height=448):
    """The numeric part of tf_hourglass_net.obj_detect_results (CenterNet/tf_hourglass_net.py:
    486-548, transpose=False): output [S, S, 4, 5 + C] -> the drawn rectangles as rows (x_lower,
    y_lower, box_width, box_height, int(100 p), class index), scale-major, np.nonzero order.
    Types as the reference's with NumPy >= 2 (NEP 50): centroid = ratio * (int64 cell + float32
    offset) * 8 in float64; size = python-float (ratio * box_scale) times a float32 output -> float32."""
    o = np.asarray(output, np.float32)
    S0, S1, ns, ch = o.shape
    n_classes = ch - 4
    w_ratio, h_ratio = img_width / img_rows, img_height / img_cols
    rows = []
    for s in range(4):
        bs = box_scales[s]
        probs = sigmoid32(o[:, :, s, 4:])
        if n_classes > 1:
            pmax, lab = probs[:, :, 1:].max(axis=2), probs[:, :, 1:].argmax(axis=2)
        else:
            pmax, lab = probs[:, :, 0], np.zeros((S0, S1), np.int64)
        xs, ys = np.nonzero(np.where(pmax >= thresh, 1, 0))
        for xi, yi in zip(xs, ys):
            b = o[xi, yi, s, :4]
            p = int(pmax[xi, yi] * np.float32(100))
            xcen = w_ratio * (float(xi) + float(b[0])) * 8
            ycen = h_ratio * (float(yi) + float(b[1])) * 8
            bw = np.float32(w_ratio * bs) * b[2]
            bh = np.float32(h_ratio * bs) * b[3]
            bw = float(img_width) if bw > img_width else float(bw)
            bh = float(img_height) if bh > img_height else float(bh)
            x_lower, y_lower = xcen - bw / 2, ycen - bh / 2
            rows.append([x_lower if x_lower >= 0 else 0.0, y_lower if y_lower >= 0 else 0.0, bw, bh, p, lab[xi, yi]])
    return np.array(rows, np.float64).reshape(-1, 6)
