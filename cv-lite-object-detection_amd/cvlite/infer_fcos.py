"""Drop-in mirror of FCOS/infer_fcos.py's numeric path on MI355X.

  image_detections(image, model, num_classes, center, iou_thresh, cls_thresh, max_detections,
                   max_total_size)                                  infer_fcos.py:27-62
runs the inference forward (BN running statistics) and one cvl_fcos_detect launch chain:
prediction_to_corners, sigmoid scores (x centerness with center=True) and
tf.image.combined_non_max_suppression, restated as HIP kernels (TF is absent from this image, so
that op's parity is pinned to the numpy restatement oracle/fcos_ref.combined_non_max_suppression,
not to TF).  Image loading / resizing (`_parse_image`, `prepare_image`) and plotting are outside
this path.  Returns the op's four outputs: (nmsed_boxes [B,T,4], nmsed_scores [B,T],
nmsed_classes [B,T], valid_detections [B]) as torch tensors on the GPU.
"""
import collections
import ctypes

import torch

from . import _lib

STRIDES = (8, 16, 32, 64, 128)

CombinedNonMaxSuppression = collections.namedtuple(
    "CombinedNonMaxSuppression", ["nmsed_boxes", "nmsed_scores", "nmsed_classes", "valid_detections"])


def detect_from_outputs(reg, cls, shapes, num_classes, center=False, iou_thresh=0.5, cls_thresh=0.05,
                        max_detections=100, max_total_size=100, strides=STRIDES):
    """Batched device form over the fused FCOS head outputs: reg [B,P,>=5] (t, b, l, r,
    centerness), cls [B,P,>=C] fp32, level shapes [(h, w)] x 5 (level-major rows)."""
    _lib.require_cuda(reg, cls)
    B, P = int(reg.shape[0]), int(reg.shape[1])
    assert sum(h * w for h, w in shapes) == P, "shapes do not match the rows"
    hw_arr = (ctypes.c_int32 * 10)(*[int(v) for hwl in shapes for v in hwl])
    st_arr = (ctypes.c_int32 * 5)(*strides)
    mpc = min(int(max_detections), P)
    T = int(max_total_size)
    dev = reg.device
    boxes = torch.empty((B, T, 4), dtype=torch.float32, device=dev)
    scores = torch.empty((B, T), dtype=torch.float32, device=dev)
    classes = torch.empty((B, T), dtype=torch.float32, device=dev)
    valid = torch.empty(B, dtype=torch.int32, device=dev)
    wsb = _lib.load().cvl_fcos_detect_workspace_size(B, P, num_classes, mpc)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    _lib.call("cvl_fcos_detect", _lib.ptr(reg.contiguous()), int(reg.shape[-1]), _lib.ptr(cls.contiguous()),
              int(cls.shape[-1]), B, ctypes.cast(hw_arr, ctypes.c_void_p), ctypes.cast(st_arr, ctypes.c_void_p),
              int(num_classes), 1 if center else 0, float(iou_thresh), float(cls_thresh), mpc, T,
              _lib.ptr(boxes), _lib.ptr(scores), _lib.ptr(classes), _lib.ptr(valid), _lib.ptr(ws), wsb,
              _lib.stream())
    return CombinedNonMaxSuppression(boxes, scores, classes, valid)


def image_detections(image, model, num_classes, center=False, iou_thresh=0.5, cls_thresh=0.05,
                     max_detections=100, max_total_size=100):
    """infer_fcos.py:27-62.  model = cvlite.fcos.build_model(...) (or its FCOSNet); image
    [B,H,W,3] / [H,W,3] fp32 (already resized and scaled to [-1, 1])."""
    net = getattr(model, "net", model)
    x = torch.as_tensor(image, dtype=torch.float32, device="cuda")
    if x.dim() == 3:
        x = x.unsqueeze(0)
    B, H, W = int(x.shape[0]), int(x.shape[1]), int(x.shape[2])
    shapes, _, _ = net.layout(B, H, W)
    reg, cls = net.forward(x.contiguous(), train=False)
    return detect_from_outputs(reg, cls, shapes, num_classes, center, iou_thresh, cls_thresh, max_detections,
                               max_total_size)
