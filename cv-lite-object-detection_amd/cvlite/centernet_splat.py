"""Drop-in mirror of CenterNet/tf_centernet.py's `format_data` (the inverse-power centre splat,
tf_centernet.py:152-342) on MI355X (cvl_centernet_splat)."""
import numpy as np
import torch

from . import _lib
from . import ops_targets as ot


def format_data(gt_labels, img_dim, num_classes, img_pad=None, stride=8, sigma=0.25):
    """-> float32 [pad_h/s, pad_w/s, 5+C] (ltrb, splat, class bits)."""
    if img_pad is None:
        img_pad = [int(float(v)) for v in np.asarray(img_dim, np.float32)]
    gt = np.asarray(gt_labels, dtype=np.float32).reshape(-1, 5)
    n = len(gt)
    boxes = np.zeros((1, max(n, 1), 5), np.float32)
    boxes[0, :n] = gt
    _lib.require_cuda()
    out = ot.centernet_splat(torch.tensor(boxes, device="cuda"), torch.tensor([n], dtype=torch.int32, device="cuda"),
                             torch.tensor(np.asarray(img_dim, np.float32).reshape(1, 2), device="cuda"),
                             (int(img_pad[0]), int(img_pad[1])), num_classes, stride=stride, sigma=sigma)
    return out[0].cpu().numpy()
