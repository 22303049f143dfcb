"""Numpy restatement of CenterNet v2's `image_augment` (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/CenterNet/train_hourglass_voc.py:24-67, called per image at :209-211 on the
padded image [N, N, 3] fp32 and its float64 target map [S, S, 4, 5 + C] (channels: 0 y offset,
1 x offset, 2 h reg, 3 w reg, 4 mask, 5.. one-hot class).  Pinned by
tests/golden/golden_image_augment.npz, which executes the reference's own `image_augment` (under
the numpy TF stub) -- see tests/golden/make_golden.py `work_image_augment`.

The branch draws are np.random.uniform() calls in the reference's order (:25, :26, :28 / :55), so
with the same numpy state the same branch is taken.  The magnitudes of brightness / contrast come
from tf.random in the reference (tf.image.random_brightness(img, 0.25): delta ~ U[-0.25, 0.25);
tf.image.random_contrast(img, 0.75, 1.25): factor ~ U[0.75, 1.25)); here they come from a second
generator so the numpy stream the rest of the training loop draws from is not shifted.

Op codes (shared with cvl_image_augment, include/cvlite.h): 0 none, 1 brightness, 2 contrast,
3 flip left-right, 4 transpose (90 degrees), 5 transpose + flip up-down (270 degrees).

The reference's transpose branch (:44-52) writes through an alias: `img_bbox = tmp_bbox` is the
same array, so `img_bbox[..., 0] = tmp_bbox[..., 1]` and then `img_bbox[..., 1] = tmp_bbox[..., 0]`
leave BOTH channels 0 and 1 equal to the transposed x offset (and 2, 3 both the w reg).  That is the
reference's behaviour and is restated as such.
"""
import numpy as np

NONE, BRIGHTNESS, CONTRAST, FLIP_LR, TRANSPOSE, ROT270 = range(6)


def draw_augment(p=0.5, rng=np.random, tf_rng=None):
    """(op, param) of one image_augment call (:25-67 control flow); rng supplies the reference's
    np.random.uniform() draws, tf_rng (default: rng) the tf.random magnitudes."""
    tf_rng = rng if tf_rng is None else tf_rng
    if rng.uniform() >= p:                                   # :25
        p_tmp = rng.uniform()                                # :26
        if p_tmp <= 0.333:
            if rng.uniform() <= 0.50:                        # :28-29
                return BRIGHTNESS, float(np.float32(tf_rng.uniform(-0.25, 0.25)))
            return CONTRAST, float(np.float32(tf_rng.uniform(0.75, 1.25)))
        if p_tmp <= 0.667:                                   # :33
            return FLIP_LR, 0.0
        return (ROT270 if rng.uniform() >= 0.50 else TRANSPOSE), 0.0     # :55-56
    return NONE, 0.0


def adjust_contrast(img, factor):
    """tf.image.adjust_contrast of one [N, N, 3] fp32 image: per-channel mean over the pixels, then
    (x - mean) * factor + mean, each op rounded to fp32.

    The mean is a RESTATEMENT: it is summed in float64 and rounded once to fp32 (as is the golden's
    numpy TF stub and cvl_image_augment's fixed-order partials), whereas TF's kernel reduces in fp32
    in its own order.  TF is not importable here, so the contrast mean's rounding is parity
    unpinned: contrast outputs are tolerance-equal (a few ulp of the mean), not bit-equal, to TF."""
    a = np.asarray(img, np.float32)
    m = a.astype(np.float64).mean(axis=(0, 1)).astype(np.float32)
    return ((a - m) * np.float32(factor) + m).astype(np.float32)


def image_augment_ref(img, bbox, op, param):
    """One image's transform for a drawn (op, param): img [N, N, 3] fp32, bbox [S, S, 4, 5+C] (its
    float64 values as the reference builds them, or fp32).  Returns new arrays (inputs untouched)."""
    img = np.asarray(img, np.float32)
    bbox = np.array(bbox, copy=True)
    if op == BRIGHTNESS:                                     # :30 (no clipping in TF2)
        return (img + np.float32(param)).astype(np.float32), bbox
    if op == CONTRAST:                                       # :32
        return adjust_contrast(img, param), bbox
    if op == FLIP_LR:                                        # :35-41
        out = bbox[:, ::-1, :, :].copy()
        out[:, :, :, 1] = 1.0 - out[:, :, :, 1]
        return np.ascontiguousarray(img[:, ::-1, :]), out
    if op in (TRANSPOSE, ROT270):                            # :44-63
        im = np.ascontiguousarray(np.transpose(img, (1, 0, 2)))
        t = np.ascontiguousarray(np.transpose(bbox, (1, 0, 2, 3)))
        t[..., 0] = t[..., 1]                                # the aliased swap (see module doc)
        t[..., 2] = t[..., 3]
        if op == ROT270:
            im = np.ascontiguousarray(im[::-1])
            t = np.ascontiguousarray(t[::-1])
            t[..., 0] = 1.0 - t[..., 0]
        return im, t
    return img.copy(), bbox
