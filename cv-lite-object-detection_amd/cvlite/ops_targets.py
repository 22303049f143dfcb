"""Device ops for target assignment and the fused detection losses (C ABI: include/cvlite.h)."""
import torch

from . import _lib
from ._lib import ptr

FCOS_STRIDES = (8, 16, 32, 64, 128)      # FCOS/fcos.py:142-143
FCOS_BOUNDS = (32.0, 64.0, 128.0, 256.0)  # FCOS/fcos.py:145-147


def fcos_level_shapes(pad_h, pad_w, strides=FCOS_STRIDES):
    return [(int(pad_h // s), int(pad_w // s)) for s in strides]


def fcos_assign(boxes, nbox, img_dim, pad_hw, num_classes, strides=FCOS_STRIDES, bounds=FCOS_BOUNDS,
                out=None, num_targets=None):
    """Batched FCOS targets.  boxes [B,Nmax,5] f32, nbox [B] i32, img_dim [B,2] f32 (device).
    Returns targets [B, P, 5+C] f32 (level-major cells) and num_targets [B,5] i32."""
    _lib.require_cuda(boxes, nbox, img_dim)
    assert boxes.dtype == torch.float32 and nbox.dtype == torch.int32 and img_dim.dtype == torch.float32
    B, nmax = int(boxes.shape[0]), int(boxes.shape[1])
    P = sum(h * w for h, w in fcos_level_shapes(pad_hw[0], pad_hw[1], strides))
    if out is None:
        out = torch.empty((B, P, 5 + num_classes), device=boxes.device, dtype=torch.float32)
    if num_targets is None:
        num_targets = torch.empty((B, 5), device=boxes.device, dtype=torch.int32)
    st = (_lib.ctypes.c_int32 * 5)(*[int(s) for s in strides])
    bd = (_lib.ctypes.c_float * 4)(*[float(x) for x in bounds])
    _lib.call("cvl_fcos_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]),
              int(pad_hw[1]), int(num_classes), _lib.ctypes.cast(st, _lib.c_void_p),
              _lib.ctypes.cast(bd, _lib.c_void_p), ptr(out), ptr(num_targets), _lib.stream())
    return out, num_targets


def fcos_center_assign(boxes, nbox, img_dim, pad_hw, num_classes, strides=FCOS_STRIDES, b_dim=FCOS_BOUNDS,
                       center_only=False, out=None, num_targets=None):
    """Batched FCOS-center targets (fcos_center.py:149-317) in cvl_fcos_assign's layout:
    targets [B, P, 5+C] f32 level-major, num_targets [B,5] i32."""
    _lib.require_cuda(boxes, nbox, img_dim)
    assert boxes.dtype == torch.float32 and nbox.dtype == torch.int32 and img_dim.dtype == torch.float32
    B, nmax = int(boxes.shape[0]), int(boxes.shape[1])
    P = sum(h * w for h, w in fcos_level_shapes(pad_hw[0], pad_hw[1], strides))
    if out is None:
        out = torch.empty((B, P, 5 + num_classes), device=boxes.device, dtype=torch.float32)
    if num_targets is None:
        num_targets = torch.empty((B, 5), device=boxes.device, dtype=torch.int32)
    st = (_lib.ctypes.c_int32 * 5)(*[int(s) for s in strides])
    bd = (_lib.ctypes.c_float * 4)(*[float(x) for x in b_dim])
    _lib.call("cvl_fcos_center_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]),
              int(pad_hw[1]), int(num_classes), _lib.ctypes.cast(st, _lib.c_void_p),
              _lib.ctypes.cast(bd, _lib.c_void_p), 1 if center_only else 0, ptr(out), ptr(num_targets),
              _lib.stream())
    return out, num_targets


def fcos_center_v1_assign(boxes, nbox, img_dim, pad_hw, num_classes, strides=FCOS_STRIDES, b_dim=FCOS_BOUNDS,
                          out=None, num_targets=None):
    """fcos_center_v1.format_data batched (cvl_fcos_center_v1_assign): centroid cells only,
    (y_off, x_off, h / box_sc, w / box_sc, 1, class bits).  Same layout as fcos_center_assign."""
    B, nmax = _boxes_args(boxes, nbox, img_dim)
    P = sum(h * w for h, w in fcos_level_shapes(pad_hw[0], pad_hw[1], strides))
    if out is None:
        out = torch.empty((B, P, 5 + num_classes), device=boxes.device, dtype=torch.float32)
    if num_targets is None:
        num_targets = torch.empty((B, 5), device=boxes.device, dtype=torch.int32)
    st = (_lib.ctypes.c_int32 * 5)(*[int(s) for s in strides])
    bd = (_lib.ctypes.c_float * 4)(*[float(x) for x in b_dim])
    _lib.call("cvl_fcos_center_v1_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]),
              int(pad_hw[1]), int(num_classes), _lib.ctypes.cast(st, _lib.c_void_p),
              _lib.ctypes.cast(bd, _lib.c_void_p), ptr(out), ptr(num_targets), _lib.stream())
    return out, num_targets


def fcos_loss(reg_pred, cls_pred, targets, num_classes, reg_type="l1", grad_scale=1.0,
              with_grad=True, grad_dtype=torch.float32, d_reg=None, d_cls=None, cen_type="l1",
              reg_sigmoid=False, cen_in_cls=False, alpha=0.25, gamma=2.0, delta=1.0, float_mask=False,
              losses=None):
    """Fused focal + smooth-L1/IoU + centerness forward and backward.
    reg_pred [B,P,ld_reg>=5] f32, cls_pred [B,P,ld_cls>=C] f32, targets [B,P,5+C] f32.
    Centre variants (fcos_center / fcos_center_v1): cen_type "focal", reg_sigmoid (v1's sigmoid
    reg head), cen_in_cls (centerness logit in class column round_up(C, 8)).
    alpha / gamma / delta: the focal_loss / smooth_l1_loss keywords (fcos.py:380, 443-444);
    float_mask: the regression mask is targets[..., 5] itself (C = 1).  losses: optional [B,3] f32
    output buffer.  Returns (losses [B,3] f32 = (cls, reg, cen) per image, d_reg, d_cls)."""
    _lib.require_cuda(reg_pred, cls_pred, targets)
    B, P = int(targets.shape[0]), int(targets.shape[1])
    assert reg_pred.shape[:2] == (B, P) and cls_pred.shape[:2] == (B, P)
    rt = reg_type if isinstance(reg_type, int) else {"l1": 0, "iou": 1}[reg_type]    # int: raw kernel flags
    rt |= (4 if cen_type.lower() == "focal" else 0) | (8 if reg_sigmoid else 0) | (16 if cen_in_cls else 0)
    rt |= 32 if float_mask else 0
    dev = targets.device
    if losses is None:
        losses = torch.empty((B, 3), device=dev, dtype=torch.float32)
    assert losses.shape == (B, 3) and losses.dtype == torch.float32 and losses.is_contiguous()
    ws = torch.empty(int(_lib.load().cvl_fcos_loss_workspace_size(B, P)), device=dev, dtype=torch.uint8)
    if with_grad:
        if d_reg is None:
            d_reg = torch.empty((B, P, reg_pred.shape[2]), device=dev, dtype=grad_dtype)
        if d_cls is None:
            d_cls = torch.empty((B, P, cls_pred.shape[2]), device=dev, dtype=grad_dtype)
    dt = lambda t: 0 if t is None or t.dtype == torch.float32 else 1  # noqa: E731
    dflt = alpha == 0.25 and gamma == 2.0 and delta == 1.0 and not float_mask
    tail = (ptr(d_reg), int(d_reg.shape[2]) if d_reg is not None else 0, dt(d_reg),
            ptr(d_cls), int(d_cls.shape[2]) if d_cls is not None else 0, dt(d_cls), ptr(ws), ws.numel(),
            _lib.stream())
    head = (ptr(reg_pred), int(reg_pred.shape[2]), ptr(cls_pred), int(cls_pred.shape[2]), ptr(targets), B, P,
            int(num_classes), rt, float(grad_scale))
    if dflt:
        _lib.call("cvl_fcos_loss", *head, ptr(losses), *tail)
    else:
        _lib.call("cvl_fcos_loss_ex", *head, float(alpha), float(gamma), float(delta), ptr(losses), *tail)
    return losses, d_reg, d_cls


def _boxes_args(boxes, nbox, img_dim):
    _lib.require_cuda(boxes, nbox, img_dim)
    assert boxes.dtype == torch.float32 and nbox.dtype == torch.int32 and img_dim.dtype == torch.float32
    return int(boxes.shape[0]), int(boxes.shape[1])


RETINA_STRIDES = (8, 16, 32, 64, 128)    # RetinaNet/retinanet_module.py:197


def retina_assign(boxes, nbox, img_dim, pad, anchor_dims, num_classes, iou_thresh=0.5,
                  strides=RETINA_STRIDES, out=None, num_targets=None):
    """Batched RetinaNet targets.  anchor_dims: device fp32 [5, A, 2].  Returns (targets
    [B, sum_l A*S_l^2, 4+C] f32 ordered (level, anchor, u, v), num_targets [B] i32)."""
    B, nmax = _boxes_args(boxes, nbox, img_dim)
    A = int(anchor_dims.shape[1])
    P = sum(A * (pad // s) ** 2 for s in strides)
    if out is None:
        out = torch.empty((B, P, 4 + num_classes), device=boxes.device, dtype=torch.float32)
    nt = torch.empty((B,), device=boxes.device, dtype=torch.int32) if num_targets is None else num_targets
    st = (_lib.ctypes.c_int32 * 5)(*[int(s) for s in strides])
    _lib.call("cvl_retina_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad), int(num_classes),
              ptr(anchor_dims.contiguous()), A, _lib.ctypes.cast(st, _lib.c_void_p), float(iou_thresh), ptr(out),
              ptr(nt), _lib.stream())
    return out, nt


def centernet_assign(boxes, nbox, img_dim, pad_hw, num_classes, stride=8, out=None):
    """CenterNet hourglass centroid targets -> [B, pad_w/s, pad_h/s, 4+C]."""
    B, nmax = _boxes_args(boxes, nbox, img_dim)
    if out is None:
        out = torch.empty((B, pad_hw[1] // stride, pad_hw[0] // stride, 4 + num_classes), device=boxes.device,
                      dtype=torch.float32)
    _lib.call("cvl_centernet_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]),
              int(pad_hw[1]), int(num_classes), int(stride), ptr(out), _lib.stream())
    return out


def centernet_splat(boxes, nbox, img_dim, pad_hw, num_classes, stride=8, sigma=0.25):
    """CenterNet centre splat targets -> [B, pad_h/s, pad_w/s, 5+C]."""
    B, nmax = _boxes_args(boxes, nbox, img_dim)
    out = torch.empty((B, pad_hw[0] // stride, pad_hw[1] // stride, 5 + num_classes), device=boxes.device,
                      dtype=torch.float32)
    _lib.call("cvl_centernet_splat", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]),
              int(pad_hw[1]), int(num_classes), int(stride), float(sigma), ptr(out), _lib.stream())
    return out


def det_loss(reg_pred, cls_pred, targets, num_classes, grad_scale_cls=1.0, grad_scale_reg=1.0, with_grad=True):
    """Focal + masked smooth-L1 (CenterNet / RetinaNet).  reg [B,P,>=4], cls [B,P,>=C], targets
    [B,P,4+C] (f32).  Returns (losses [B,2] = (cls, reg), d_reg, d_cls)."""
    _lib.require_cuda(reg_pred, cls_pred, targets)
    B, P = int(targets.shape[0]), int(targets.shape[1])
    dev = targets.device
    losses = torch.empty((B, 2), device=dev, dtype=torch.float32)
    ws = torch.empty(int(_lib.load().cvl_det_loss_workspace_size(B, P)), device=dev, dtype=torch.uint8)
    d_reg = torch.zeros_like(reg_pred) if with_grad else None
    d_cls = torch.zeros_like(cls_pred) if with_grad else None
    _lib.call("cvl_det_loss", ptr(reg_pred), int(reg_pred.shape[-1]), ptr(cls_pred), int(cls_pred.shape[-1]),
              ptr(targets), B, P, int(num_classes), float(grad_scale_cls), float(grad_scale_reg), ptr(losses),
              ptr(d_reg), ptr(d_cls), ptr(ws), _lib.stream())
    return losses, d_reg, d_cls


def retina_loss(reg_pred, cls_pred, targets, level_cells, n_anchors, num_classes, img_weight=None,
                grad_scale=1.0, d_reg=None, d_cls=None, losses=None):
    """RetinaNet.train_loss fwd+bwd (cvl_retina_loss).  reg_pred [B,P,ld>=4A] / cls_pred [B,P,ld>=AC] f32
    from the grouped heads, targets [B, A*P, 4+C] (cvl_retina_assign order).  d_reg / d_cls: bf16
    (fp32 in the parity mode) buffers written at the prediction positions (None = no gradient).
    Returns losses [B,2]."""
    _lib.require_cuda(reg_pred, cls_pred, targets)
    B, P = int(reg_pred.shape[0]), int(reg_pred.shape[1])
    assert sum(level_cells) == P and int(targets.shape[1]) == n_anchors * P
    dev = targets.device
    if losses is None:
        losses = torch.empty((B, 2), device=dev, dtype=torch.float32)
    ws = torch.empty(int(_lib.load().cvl_retina_loss_workspace_size(B, P, n_anchors)), device=dev, dtype=torch.uint8)
    lc = (_lib.ctypes.c_int32 * 5)(*[int(c) for c in level_cells])
    f32 = any(t is not None and t.dtype == torch.float32 for t in (d_reg, d_cls))    # fp32 parity mode
    for t in (d_reg, d_cls):
        assert t is None or t.dtype == (torch.float32 if f32 else torch.bfloat16)
    _lib.call("cvl_retina_loss_f32" if f32 else "cvl_retina_loss", ptr(reg_pred), int(reg_pred.shape[-1]), ptr(cls_pred), int(cls_pred.shape[-1]),
              ptr(targets), B, _lib.ctypes.cast(lc, _lib.c_void_p), int(n_anchors), int(num_classes), ptr(img_weight),
              float(grad_scale), ptr(losses), ptr(d_reg), int(d_reg.shape[-1]) if d_reg is not None else 0,
              ptr(d_cls), int(d_cls.shape[-1]) if d_cls is not None else 0, ptr(ws), _lib.stream())
    return losses


def nms(boxes_xyxy, classes, iou_threshold):
    """boxes [n, 6] float64 (x1, y1, x2, y2, score, cls) device; classes: iterable of class values
    in processing order.  Returns the kept rows in the reference's emission order."""
    _lib.require_cuda(boxes_xyxy)
    n = int(boxes_xyxy.shape[0])
    cls = torch.tensor(list(classes), dtype=torch.float64, device=boxes_xyxy.device)
    ncls = int(cls.numel())
    keep = torch.empty((ncls, n), dtype=torch.int32, device=boxes_xyxy.device)
    nkeep = torch.empty((ncls,), dtype=torch.int32, device=boxes_xyxy.device)
    ws = torch.empty(int(_lib.load().cvl_nms_workspace_size(n, ncls)), dtype=torch.uint8, device=boxes_xyxy.device)
    _lib.call("cvl_nms", ptr(boxes_xyxy), n, ptr(cls), ncls, float(iou_threshold), ptr(keep), ptr(nkeep),
              ptr(ws), _lib.stream())
    nk = nkeep.cpu().tolist()
    idx = torch.cat([keep[c, :nk[c]] for c in range(ncls)]) if ncls else keep.new_zeros(0)
    return boxes_xyxy[idx.long()]


def soft_nms(boxes_xyxy, classes, sigma=0.3):
    """Soft-NMS (cvl_soft_nms): boxes [n, 6] float64 (x1, y1, x2, y2, score, cls) device, classes in
    processing order.  Returns the emitted rows (reference order) with their decayed scores."""
    _lib.require_cuda(boxes_xyxy)
    n = int(boxes_xyxy.shape[0])
    dev = boxes_xyxy.device
    cls = torch.tensor(list(classes), dtype=torch.float64, device=dev)
    ncls = int(cls.numel())
    keep = torch.empty((ncls, n), dtype=torch.int32, device=dev)
    ksc = torch.empty((ncls, n), dtype=torch.float64, device=dev)
    nkeep = torch.empty((ncls,), dtype=torch.int32, device=dev)
    ws = torch.empty(int(_lib.load().cvl_soft_nms_workspace_size(n, ncls)), dtype=torch.uint8, device=dev)
    _lib.call("cvl_soft_nms", ptr(boxes_xyxy), n, ptr(cls), ncls, float(sigma), ptr(keep), ptr(ksc), ptr(nkeep),
              ptr(ws), _lib.stream())
    nk = nkeep.cpu().tolist()
    idx = torch.cat([keep[c, :nk[c]] for c in range(ncls)]).long()
    rows = boxes_xyxy[idx].clone()
    rows[:, 4] = torch.cat([ksc[c, :nk[c]] for c in range(ncls)])
    return rows


def centernet_loss(pred, targets, num_classes, cls_scale=2.5, reg_scale=1.0, d_pred=None, losses=None):
    """CenterNet model_loss fwd+bwd (tf_centernet_hourglass.py:492-505 in train_step :537-549) off
    the output conv.  pred [B,P,ld] f32 (reg 0..3, cls 4..), targets [B,P,4+C] f32.
    Returns (losses [B,2] = (cls, reg), d_pred bf16 [B,P,ld_d] of cls_scale*cls + reg_scale*reg)."""
    _lib.require_cuda(pred, targets)
    B, P = int(targets.shape[0]), int(targets.shape[1])
    dev = targets.device
    if losses is None:
        losses = torch.empty((B, 2), device=dev, dtype=torch.float32)
    if d_pred is None:
        d_pred = torch.empty((B, P, (4 + num_classes + 7) // 8 * 8), device=dev, dtype=torch.bfloat16)
    ws = torch.empty(int(_lib.load().cvl_det_loss_workspace_size(B, P)), device=dev, dtype=torch.uint8)
    _lib.call("cvl_centernet_loss", ptr(pred), int(pred.shape[-1]), ptr(targets), B, P, int(num_classes),
              float(cls_scale), float(reg_scale), ptr(losses), ptr(d_pred), int(d_pred.shape[-1]), ptr(ws),
              _lib.stream())
    return losses, d_pred


def hourglass_v2_assign(boxes, nbox, raw_dims, img_dims, num_classes, out=None):
    """CenterNet v2 targets of one batch (train_hourglass_voc.py train() :96-160): boxes [B,n_max,5]
    f32 = dataset corner rows + label, nbox [B] i32; returns [B, S, S, 4, 5+C] f32, S = img_dims/8."""
    _lib.require_cuda(boxes, nbox)
    assert boxes.dtype == torch.float32 and nbox.dtype == torch.int32
    B, nmax = int(boxes.shape[0]), int(boxes.shape[1])
    S = int(img_dims) // 8
    if out is None:
        out = torch.empty((B, S, S, 4, 5 + num_classes), device=boxes.device, dtype=torch.float32)
    assert tuple(out.shape) == (B, S, S, 4, 5 + num_classes) and out.is_contiguous()
    _lib.call("cvl_hourglass_v2_assign", ptr(boxes), ptr(nbox), B, nmax, int(raw_dims), int(img_dims),
              int(num_classes), ptr(out), _lib.stream())
    return out


def hourglass_v2_loss(pred, targets, num_classes, loss_type="focal", cls_scale=2.5, reg_scale=1.0, d_pred=None,
                      losses=None, reg_is_prob=False):
    """CenterNet v2 model_loss fwd+bwd (tf_hourglass_net.py:398-413 in train_step :415-447) off the
    head conv.  pred [B,P,ld] f32 (channel sc*(5+C)+j, b_focal folded), targets [B,P,4,5+C] f32.
    reg_is_prob: pred's box channels are the model's sigmoid outputs (model_loss's `outputs`).
    Returns (losses [B,2] = (cls, reg), d_pred bf16 [B,P,ld_d] of cls_scale*cls + reg_scale*reg)."""
    _lib.require_cuda(pred, targets)
    B, P = int(targets.shape[0]), int(targets.shape[1])
    assert tuple(targets.shape[2:]) == (4, 5 + num_classes) and pred.shape[:2] == (B, P)
    dev = targets.device
    if losses is None:
        losses = torch.empty((B, 2), device=dev, dtype=torch.float32)
    if d_pred is None:
        d_pred = torch.empty((B, P, (4 * (5 + num_classes) + 31) // 32 * 32), device=dev, dtype=torch.bfloat16)
    ws = torch.empty(int(_lib.load().cvl_hourglass_v2_loss_workspace_size(B, P)), device=dev, dtype=torch.uint8)
    lt = (1 if loss_type == "sigmoid" else 0) | (2 if reg_is_prob else 0)
    _lib.call("cvl_hourglass_v2_loss", ptr(pred), int(pred.shape[-1]), ptr(targets), B, P, int(num_classes), lt,
              float(cls_scale), float(reg_scale), ptr(losses), ptr(d_pred), int(d_pred.shape[-1]), ptr(ws),
              _lib.stream())
    return losses, d_pred


def centernet_s8_assign(boxes, nbox, img_dim, pad_hw, num_classes, box_scales, stride=8, out=None):
    """tf_centernet_resnet_s8.format_data batched (cvl_centernet_s8_assign): boxes [B,n_max,5]
    normalised (y, x, h, w, cls), img_dim [B,2] the resized size, pad_hw the padded size.
    Returns [B, pad_w/stride, pad_h/stride, n_scales, 4+C] f32."""
    B, nmax = _boxes_args(boxes, nbox, img_dim)
    ns = len(box_scales)
    hm, wm = int(pad_hw[1] / stride), int(pad_hw[0] / stride)
    if out is None:
        out = torch.empty((B, hm, wm, ns, 4 + num_classes), device=boxes.device, dtype=torch.float32)
    assert tuple(out.shape) == (B, hm, wm, ns, 4 + num_classes) and out.is_contiguous()
    sc = (_lib.ctypes.c_float * ns)(*[float(v) for v in box_scales])
    _lib.call("cvl_centernet_s8_assign", ptr(boxes), ptr(nbox), ptr(img_dim), B, nmax, int(pad_hw[0]), int(pad_hw[1]),
              int(num_classes), _lib.ctypes.cast(sc, _lib.c_void_p), ns, int(stride), ptr(out), _lib.stream())
    return out


def centernet_s8_loss(reg, cls, targets, num_classes, n_scales, cls_scale=1.0, reg_scale=1.0, d_reg=None,
                      d_cls=None, losses=None):
    """tf_centernet_resnet_s8.model_loss fwd+bwd off the two head convs: reg [B,P,>=ns*4], cls
    [B,P,>=ns*C] f32 raw logits, targets [B,P,ns,4+C].  Returns (losses [B,2], d_reg, d_cls) with
    bf16 gradients of cls_scale*cls + reg_scale*reg."""
    _lib.require_cuda(reg, cls, targets)
    B, P = int(targets.shape[0]), int(targets.shape[1])
    assert tuple(targets.shape[2:]) == (n_scales, 4 + num_classes)
    dev = targets.device
    if losses is None:
        losses = torch.empty((B, 2), device=dev, dtype=torch.float32)
    if d_reg is None:
        d_reg = torch.empty((B, P, (4 * n_scales + 31) // 32 * 32), device=dev, dtype=torch.bfloat16)
    if d_cls is None:
        d_cls = torch.empty((B, P, (num_classes * n_scales + 31) // 32 * 32), device=dev, dtype=torch.bfloat16)
    ws = torch.empty(int(_lib.load().cvl_centernet_s8_loss_workspace_size(B, P, n_scales)), device=dev,
                     dtype=torch.uint8)
    _lib.call("cvl_centernet_s8_loss", ptr(reg), int(reg.shape[-1]), ptr(cls), int(cls.shape[-1]), ptr(targets), B, P,
              int(n_scales), int(num_classes), float(cls_scale), float(reg_scale), ptr(losses), ptr(d_reg),
              int(d_reg.shape[-1]), ptr(d_cls), int(d_cls.shape[-1]), ptr(ws), _lib.stream())
    return losses, d_reg, d_cls
