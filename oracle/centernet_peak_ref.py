"""Numpy restatement of the CenterNet 3x3 max-pool peak decode (TEST INFRASTRUCTURE).

The BASELINE north_star names a "3x3 max-pool peak decode"; the reference's own CenterNet decode is
threshold + NMS (/root/reference/CenterNet/tf_centernet_hourglass.py:566-656), so this op has NO
reference implementation: parity unpinned at the reference level, pinned here by a restatement of
the standard CenterNet rule and hand-made known answers (tests/test_oracle_golden.py).
Box corners follow prediction_to_corners (tf_centernet_hourglass.py:355-377) in fp32.
"""
import numpy as np

f32 = np.float32


def sigmoid32(v):
    """float64 sigmoid rounded to fp32 (the kernel's formula)."""
    return (1.0 / (1.0 + np.exp(-np.asarray(v, np.float64)))).astype(f32)


def maxpool3x3(p):
    """[H, W, C] -> 3x3 / stride 1 max-pool with -inf padding."""
    H, W, C = p.shape
    q = np.full((H + 2, W + 2, C), -np.inf, np.float32)
    q[1:-1, 1:-1] = p
    out = np.full_like(p, -np.inf)
    for dy in range(3):
        for dx in range(3):
            out = np.maximum(out, q[dy:dy + H, dx:dx + W])
    return out


def peak_decode(pred, num_classes, stride, thresh, K):
    """pred [H, W, ld] fp32 -> rows [n <= K, 6] float64 (y_lo, x_lo, y_hi, x_hi, prob, class)."""
    pred = np.asarray(pred, np.float32)
    H, W = pred.shape[:2]
    C = num_classes
    prob = sigmoid32(pred[..., 4:4 + C])
    keep = (prob == maxpool3x3(prob)) & (prob >= f32(thresh))
    cells, cls = np.nonzero(keep.reshape(H * W, C))
    flat = cells.astype(np.int64) * C + cls
    p = prob.reshape(H * W, C)[cells, cls]
    order = np.lexsort((flat, -p.astype(np.float64)))[:K]       # prob desc, then flat index asc
    rows = np.zeros((len(order), 6), np.float64)
    st = f32(stride)
    for r, j in enumerate(order):
        cell, c = int(cells[j]), int(cls[j])
        y, x = divmod(cell, W)
        q = pred[y, x]
        gy, gx = f32(y) + f32(0.5), f32(x) + f32(0.5)
        rows[r] = [st * (gy - q[0]), st * (gx - q[2]), st * (gy + q[1]), st * (gx + q[3]), p[j], c]
    return rows
