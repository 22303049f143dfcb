"""GPU parity of the CenterNet 3x3 max-pool peak decode (cvl_centernet_peak_decode) against its numpy
restatement (oracle/centernet_peak_ref.py): peaks, order, classes and scores exact, corners fp32.
No reference implementation exists (tf_centernet_hourglass.py:566-656 decodes by threshold + NMS),
so parity is unpinned at the reference level."""
import numpy as np
import pytest
import torch

from oracle.centernet_peak_ref import peak_decode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H,W,C,thresh,K,quant", [
    (3, 17, 23, 20, 0.3, 100, False),
    (2, 32, 32, 3, 0.05, 40, True),        # quantised logits: many exact plateau ties, K cut
    (8, 128, 128, 20, 0.3, 100, False),    # CenterNet bench geometry (512 / stride 4 ... 128x128)
    (1, 4, 4, 1, 0.0, 100, False),         # every local max kept
])
def test_peak_decode_matches_restatement(B, H, W, C, thresh, K, quant):
    from cvlite.centernet_hourglass import peak_detections
    rng = np.random.default_rng(B * 1000 + H + C)
    pred = np.zeros((B, H, W, 4 + C + 3), np.float32)            # ld > 4 + C (padded channels)
    pred[..., :4] = rng.uniform(0.0, 6.0, (B, H, W, 4))
    logits = rng.normal(-2.0, 2.0, (B, H, W, C))
    if quant:
        logits = np.round(logits * 2) / 2
    pred[..., 4:4 + C] = logits
    pred[..., 4 + C:] = 99.0                                      # must be ignored
    got = peak_detections(torch.from_numpy(pred).cuda(), thresh=thresh, K=K, downsample=4, num_classes=C)
    assert len(got) == B
    for b in range(B):
        ref = peak_decode(pred[b, ..., :4 + C], C, 4, thresh, K)
        assert got[b].shape == ref.shape, (b, got[b].shape, ref.shape)
        np.testing.assert_array_equal(got[b][:, 5], ref[:, 5])
        np.testing.assert_array_equal(got[b][:, 4], ref[:, 4])
        np.testing.assert_array_equal(got[b][:, :4], ref[:, :4])
