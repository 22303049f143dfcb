"""Drop-in mirror of FCOS/data_preprocess.py's image path on MI355X.

  random_flip_horizontal(image, boxes, p_flip=0.5)                  data_preprocess.py:24-39
  resize_and_pad_image(image, jitter, min_side, max_side, stride, equal_dims)   :41-96
  preprocess_image(image, ..., flip, out)                           fused flip + resize + pad
  preprocess_data(sample)                                           :98-133 (one training sample)
  box_targets(bbox, flip)                                           flip + swap_xy + convert_to_xywh

The resize / normalise / pad (and the flip, when fused) run in one cvl_resize_pad_normalize
launch per image that can write straight into a slot of the device batch.  JPEG decode
(`_parse_image`, data_preprocess.py:5-9) is a host step (PIL's libjpeg; this ROCm image ships no
rocJPEG / GPU JPEG decoder), as the reference's tf.image.decode_jpeg runs on the host CPU too;
everything after it runs on the GPU.  The jitter draw uses numpy's generator instead of
tf.random.uniform (a different stream by construction).
"""
import numpy as np
import torch

from . import _lib

f32 = np.float32


def _plan(H, W, jitter, min_side, max_side, stride, equal_dims, rng):
    shape = np.array([H, W], f32)
    if jitter is not None:
        rng = rng if rng is not None else np.random.default_rng()
        min_side = f32(rng.uniform(jitter[0], jitter[1]))
    ratio = f32(min_side) / shape.min()
    if ratio * shape.max() > f32(max_side):
        ratio = f32(max_side) / shape.max()
    new_shape = (ratio * shape).astype(f32)
    pd = (np.ceil(new_shape / f32(stride)) * f32(stride)).astype(np.int32)
    if equal_dims:
        pd = np.array([pd.max(), pd.max()], np.int32)
    return new_shape, ratio, int(pd[0]), int(pd[1])


def preprocess_image(image, jitter=None, min_side=800.0, max_side=1333.0, stride=128.0, equal_dims=True,
                     flip=False, out=None, rng=None):
    """Fused flip + resize_and_pad_image: returns (padded [Hp,Wp,C] fp32 on the GPU, new_shape, ratio).
    out: an optional preallocated [Hp,Wp,C] fp32 slot (e.g. batch[i])."""
    _lib.require_cuda()
    img = torch.as_tensor(image).cuda()
    if img.dtype not in (torch.uint8, torch.float32):
        img = img.float()
    img = img.contiguous()
    H, W, C = int(img.shape[0]), int(img.shape[1]), int(img.shape[2])
    new_shape, ratio, ph, pw = _plan(H, W, jitter, min_side, max_side, stride, equal_dims, rng)
    oh, ow = int(new_shape[0]), int(new_shape[1])
    if out is None:
        out = torch.empty((ph, pw, C), dtype=torch.float32, device=img.device)
    assert tuple(out.shape) == (ph, pw, C) and out.dtype == torch.float32 and out.is_contiguous()
    _lib.call("cvl_resize_pad_normalize", _lib.ptr(img), 1 if img.dtype == torch.uint8 else 0, H, W, C,
              1 if flip else 0, oh, ow, ph, pw, _lib.ptr(out), _lib.stream())
    return out, new_shape, ratio


def resize_and_pad_image(image, jitter=[640, 1024], min_side=800.0, max_side=1333.0, stride=128.0,
                         equal_dims=True):
    """data_preprocess.py:41-96 -> (image_padded, new_shape, ratio)."""
    return preprocess_image(image, jitter, min_side, max_side, stride, equal_dims)


def random_flip_horizontal(image, boxes, p_flip=0.5, rng=None):
    """data_preprocess.py:24-39: with probability p_flip, flip the image left-right and map the
    normalised boxes [x1, y1, x2, y2] -> [1 - x2, y1, 1 - x1, y2]."""
    rng = rng if rng is not None else np.random.default_rng()
    if rng.uniform() <= p_flip:
        _lib.require_cuda()
        img = torch.as_tensor(image).cuda()
        b = np.asarray(boxes, f32)
        return torch.flip(img, dims=[1]), np.stack([f32(1.0) - b[:, 2], b[:, 1], f32(1.0) - b[:, 0], b[:, 3]], -1)
    return image, boxes


def _parse_image(filename):
    """data_preprocess.py:5-9 `_parse_image`: read + decode a JPEG/PNG file to an [H,W,3] uint8
    array (host; PIL's libjpeg decode with its default islow IDCT, where the reference uses
    tf.image.decode_jpeg -- parity unpinned at the pixel level, TF absent).  The decoded image
    then goes to the GPU resize / pad kernel."""
    from PIL import Image
    with Image.open(filename) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def box_targets(bbox, flip):
    """The box half of preprocess_data (data_preprocess.py:120-131) in the reference's fp32 order:
    random_flip_horizontal's box map [b0, b1, b2, b3] -> [1-b2, b1, 1-b0, b3] when flipped
    (:36-39), utils.swap_xy (:5-13), utils.convert_to_xywh (:15-27)."""
    b = np.asarray(bbox, f32).reshape(-1, 4)
    if flip:
        b = np.stack([f32(1.0) - b[:, 2], b[:, 1], f32(1.0) - b[:, 0], b[:, 3]], -1)
    s = np.stack([b[:, 1], b[:, 0], b[:, 3], b[:, 2]], -1)
    return np.concatenate([(s[:, :2] + s[:, 2:]) / f32(2.0), s[:, 2:] - s[:, :2]], -1).astype(f32)


def preprocess_data(sample, img_dims=384, pad_flag=True, rng=None, out=None):
    """data_preprocess.py:98-133 preprocess_data(sample, img_dims, pad_flag) for one sample dict with
    the reference's keys: image (a file name, decoded on the host by _parse_image, or an already
    decoded [H,W,3] image, uint8 or fp32, host or device), objects = {bbox [N,4] normalised, label
    [N]}, l_jitter / u_jitter, min_side, max_side.  Returns (image [Hp,Wp,3] fp32 on the GPU, bbox
    [N,4] (the reference's xywh of the swapped corners), class_id [N] int32, img_shp [2] fp32).
    pad_flag=True: flip + jittered resize_and_pad_image (img_shp = the unpadded resized shape);
    pad_flag=False: resize to [img_dims, img_dims] (:111-113), flip, /127.5 - 1 (:124-125),
    img_shp = [img_dims, img_dims] -- one fused launch either way, in the reference's order (pad_flag
    True: flip, then resize; False: resize, then flip its output).  The flip draw (p = 0.5) and the jitter draw use `rng`
    (numpy) in the reference's order: flip first, then the jitter size."""
    rng = rng if rng is not None else np.random.default_rng()
    jitter = [sample["l_jitter"], sample["u_jitter"]]
    image = sample["image"]
    if isinstance(image, str):                   # a file name, as the reference's samples hold
        image = _parse_image(image)
    flip = bool(rng.uniform() <= 0.5)
    if pad_flag:
        img, new_shape, _ = preprocess_image(image, jitter=jitter, min_side=sample["min_side"],
                                             max_side=sample["max_side"], flip=flip, out=out, rng=rng)
    else:
        img = resize_normalize(image, int(img_dims), int(img_dims), flip=flip, out=out, flip_after=True)
        new_shape = np.array([img_dims, img_dims], f32)
    bbox = box_targets(sample["objects"]["bbox"], flip)
    cls = np.asarray(sample["objects"]["label"], np.int32).reshape(-1)
    return img, bbox, cls, np.asarray(new_shape, f32)


def resize_normalize(image, oh, ow, flip=False, out=None, flip_after=False):
    """tf.image.resize(image, [oh, ow]) (bilinear, half-pixel) [+ flip_left_right of the input, or of
    the resized output with flip_after], / 127.5 - 1, no padding: one cvl_resize_pad_normalize launch
    (output size = padded size)."""
    _lib.require_cuda()
    img = torch.as_tensor(image).cuda()
    if img.dtype not in (torch.uint8, torch.float32):
        img = img.float()
    img = img.contiguous()
    H, W, C = int(img.shape[0]), int(img.shape[1]), int(img.shape[2])
    if out is None:
        out = torch.empty((oh, ow, C), dtype=torch.float32, device=img.device)
    assert tuple(out.shape) == (oh, ow, C) and out.dtype == torch.float32 and out.is_contiguous()
    _lib.call("cvl_resize_pad_normalize", _lib.ptr(img), 1 if img.dtype == torch.uint8 else 0, H, W, C,
              (2 if flip_after else 1) if flip else 0, oh, ow, oh, ow, _lib.ptr(out), _lib.stream())
    return out


def padded_size(sample_hw, jitter, min_side, max_side, rng, stride=128.0):
    """Host-only size plan of preprocess_data (the padded square side and new_shape) for the same
    rng draw order (flip, then jitter): used to bucket a batch before any image moves."""
    flip = bool(rng.uniform() <= 0.5)
    new_shape, _, ph, pw = _plan(sample_hw[0], sample_hw[1], jitter, min_side, max_side, stride, True, rng)
    return flip, new_shape, ph
