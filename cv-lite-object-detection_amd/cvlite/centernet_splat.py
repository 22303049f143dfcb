"""Drop-in mirror of CenterNet/tf_centernet.py on MI355X: `format_data` (the inverse-power centre
splat, tf_centernet.py:152-342; cvl_centernet_splat) and `center_dist_1d` / `center_dist_2d`
(:6-19; cvl_center_dist)."""
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


def _center_dist(grid_x, grid_y, mu_x, mu_y, spread):
    gx = np.asarray(grid_x, np.float64)
    _lib.require_cuda()
    x = torch.tensor(gx.reshape(-1), device="cuda")
    y = torch.tensor(np.asarray(grid_y, np.float64).reshape(-1), device="cuda") if grid_y is not None else None
    out = torch.empty_like(x)
    _lib.call("cvl_center_dist", _lib.ptr(x), _lib.ptr(y), int(x.numel()), float(mu_x), float(mu_y), float(spread),
              _lib.ptr(out), _lib.stream())
    return out.cpu().numpy().reshape(gx.shape)


def center_dist_1d(grid_x, mu_x=0.0, spread=2.0):
    """tf_centernet.py:6-10: 1 / (x - mu_x)^spread normalised by its maximum."""
    return _center_dist(grid_x, None, mu_x, 0.0, spread)


def center_dist_2d(grid_x, grid_y, mu_x=0.0, mu_y=0.0, spread=2.0):
    """tf_centernet.py:12-19: the product of the two inverse powers, normalised by its maximum."""
    return _center_dist(grid_x, grid_y, mu_x, mu_y, spread)
