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
