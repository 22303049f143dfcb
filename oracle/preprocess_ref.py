"""Numpy restatement of the FCOS input pipeline (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/FCOS/data_preprocess.py:24-133 (`random_flip_horizontal`,
`resize_and_pad_image`).  The resize is TF2's `tf.image.resize(method="bilinear")` (half-pixel
centres, antialias off) restated from TF's published kernel in fp32 — TF is not installed here, so
this restatement is pinned by known answers (identity at equal size, 2x2 means at exact 2x
downscale, edge clamping), not by TF itself: parity unpinned at the TF level.
"""
import numpy as np

f32 = np.float32


def _weights(out_size, in_size):
    scale = f32(in_size) / f32(out_size)
    o = np.arange(out_size, dtype=f32)
    v = (o + f32(0.5)) * scale - f32(0.5)
    fl = np.floor(v)
    lo = np.maximum(fl.astype(np.int64), 0)
    hi = np.minimum(np.ceil(v).astype(np.int64), in_size - 1)
    return lo, hi, (v - fl).astype(f32)


def resize_bilinear(img, out_h, out_w):
    """tf.image.resize(img [H,W,C], [out_h, out_w]) -> fp32 (half-pixel, no antialias)."""
    a = np.asarray(img).astype(f32)
    H, W = a.shape[:2]
    y0, y1, yl = _weights(out_h, H)
    x0, x1, xl = _weights(out_w, W)
    tl, tr = a[y0][:, x0], a[y0][:, x1]
    bl, br = a[y1][:, x0], a[y1][:, x1]
    xl = xl[None, :, None]
    yl = yl[:, None, None]
    top = tl + (tr - tl) * xl
    bot = bl + (br - bl) * xl
    return (top + (bot - top) * yl).astype(f32)


def flip_boxes(boxes):
    """random_flip_horizontal's box update (data_preprocess.py:36-38), normalised corners."""
    b = np.asarray(boxes, f32)
    return np.stack([f32(1.0) - b[:, 2], b[:, 1], f32(1.0) - b[:, 0], b[:, 3]], -1)


def resize_and_pad_image(image, min_side=800.0, max_side=1333.0, stride=128.0, equal_dims=True, flip=False):
    """data_preprocess.py:41-96 with jitter resolved by the caller (min_side given):
    -> (padded fp32 image, new_shape fp32 [2], ratio fp32)."""
    a = np.asarray(image)
    if flip:
        a = a[:, ::-1]
    shape = np.array(a.shape[:2], f32)
    ratio = f32(min_side) / shape.min()
    if ratio * shape.max() > f32(max_side):
        ratio = f32(max_side) / shape.max()
    new_shape = (ratio * shape).astype(f32)
    oh, ow = int(new_shape[0]), int(new_shape[1])
    r = resize_bilinear(a, oh, ow) / f32(127.5) - f32(1.0)
    pd = (np.ceil(new_shape / f32(stride)) * f32(stride)).astype(np.int32)
    if equal_dims:
        pd = np.array([pd.max(), pd.max()])
    out = np.zeros((int(pd[0]), int(pd[1]), a.shape[2]), f32)
    out[:oh, :ow] = r
    return out, new_shape, ratio
