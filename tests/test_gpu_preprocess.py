"""GPU parity of the input pipeline kernel (FCOS/data_preprocess.py:24-133): cvl_resize_pad_normalize
vs the numpy restatement oracle/preprocess_ref (bit-exact: the same fp32 operation sequence), for
uint8 and fp32 sources, down- and up-scaling, flip, jitter-style odd sizes and padding.  The TF
resize itself is not installed: parity is pinned to the restatement (known answers in
tests/test_oracle_golden.py), not to TF."""
import numpy as np
import pytest
import torch

from oracle import preprocess_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W,min_side,max_side,flip,u8", [
    (375, 500, 512.0, 512.0, False, True),     # VOC-sized photo, the bench's fixed 512 input
    (500, 333, 640.0, 1024.0, True, True),
    (480, 640, 800.0, 1333.0, False, False),
    (1024, 768, 417.3, 600.0, True, False),    # downscale, odd jittered side
    (64, 64, 64.0, 64.0, False, True),         # same size: identity up to the normalisation
])
def test_resize_pad_vs_restatement(H, W, min_side, max_side, flip, u8):
    from cvlite.data_preprocess import preprocess_image
    rng = np.random.default_rng(H * 7 + W)
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    src = img if u8 else img.astype(np.float32) + rng.uniform(0, 1, img.shape).astype(np.float32)
    got, ns, ratio = preprocess_image(src, None, min_side, max_side, 128.0, True, flip=flip)
    ref, rns, rratio = preprocess_ref.resize_and_pad_image(src, min_side, max_side, 128.0, True, flip=flip)
    np.testing.assert_array_equal(ns, rns)
    assert ratio == rratio
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_batch_slot_and_flip_boxes():
    from cvlite.data_preprocess import preprocess_image, random_flip_horizontal
    rng = np.random.default_rng(0)
    batch = torch.zeros((2, 512, 512, 3), device="cuda")
    imgs = [rng.integers(0, 256, (300 + 50 * i, 400, 3), dtype=np.uint8) for i in range(2)]
    for i, im in enumerate(imgs):
        preprocess_image(im, None, 512.0, 512.0, 128.0, True, out=batch[i])
        ref = preprocess_ref.resize_and_pad_image(im, 512.0, 512.0, 128.0, True)[0]
        np.testing.assert_array_equal(batch[i].cpu().numpy(), ref)
    boxes = np.array([[0.1, 0.2, 0.5, 0.9]], np.float32)
    im2, b2 = random_flip_horizontal(torch.tensor(imgs[0]).cuda(), boxes, p_flip=1.0)
    np.testing.assert_array_equal(im2.cpu().numpy(), imgs[0][:, ::-1])
    np.testing.assert_array_equal(b2, preprocess_ref.flip_boxes(boxes))


def test_preprocess_data_from_jpeg_file(tmp_path):
    """data_preprocess.preprocess_data on a sample whose image is a JPEG FILE NAME (the reference's
    VOC sample schema, data_preprocess.py:5-9 _parse_image -> :98-133): host decode (PIL) then the
    fused GPU flip + resize + pad -- identical to the restatement on the same decoded pixels and
    the same flip / jitter draws; and the pad_flag=False form (resize to img_dims, flip, /127.5-1)."""
    from PIL import Image
    from cvlite.data_preprocess import preprocess_data, _parse_image
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (333, 500, 3), dtype=np.uint8)
    path = str(tmp_path / "sample.jpg")
    Image.fromarray(img).save(path, quality=90)
    dec = _parse_image(path)
    assert dec.shape == (333, 500, 3) and dec.dtype == np.uint8
    sample = {"image": path, "objects": {"bbox": np.array([[0.1, 0.2, 0.6, 0.9]], np.float32),
                                         "label": np.array([3], np.int32)},
              "l_jitter": 480, "u_jitter": 544, "min_side": 512.0, "max_side": 512.0}
    for seed in (0, 1, 2, 3):
        out, bbox, cls, shp = preprocess_data(sample, rng=np.random.default_rng(seed))
        r = np.random.default_rng(seed)
        flip = bool(r.uniform() <= 0.5)
        side = np.float32(r.uniform(480, 544))
        ref, rns, _ = preprocess_ref.resize_and_pad_image(dec, side, 512.0, 128.0, True, flip=flip)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        np.testing.assert_array_equal(shp, rns)
        assert cls.tolist() == [3]
        b = preprocess_ref.flip_boxes(sample["objects"]["bbox"]) if flip else sample["objects"]["bbox"]
        np.testing.assert_allclose(bbox, [[(b[0, 1] + b[0, 3]) / 2, (b[0, 0] + b[0, 2]) / 2,
                                           b[0, 3] - b[0, 1], b[0, 2] - b[0, 0]]], rtol=1e-6)
        # pad_flag=False: tf.image.resize to img_dims, then the flip, then /127.5 - 1
        out2, _, _, shp2 = preprocess_data(sample, img_dims=384, pad_flag=False, rng=np.random.default_rng(seed))
        rf = preprocess_ref.resize_bilinear(dec, 384, 384)                 # the reference's order:
        rf = (rf[:, ::-1] if flip else rf) / np.float32(127.5) - np.float32(1.0)   # resize, flip, scale
        np.testing.assert_array_equal(out2.cpu().numpy(), rf)
        np.testing.assert_array_equal(shp2, [384.0, 384.0])
