"""torch-CPU float64 restatement of FCOS/fcos.py:380-496 with autograd (TEST INFRASTRUCTURE):
the gradient oracle for the fused loss kernel (the TF GradientTape of the reference cannot run
here).  Forward values are pinned to the reference goldens through oracle/fcos_ref.py."""
import torch


def focal(y, x, alpha=0.25):
    L = torch.log1p(torch.exp(-x.abs()))
    p = torch.sigmoid(x)
    return (y * alpha * L * (1 - p) ** 2 + p ** 2 * (1 - y) * (1 - alpha) * L
            + (1 - y) * (1 - alpha) * torch.clamp(x, min=0) * p ** 2
            - y * alpha * torch.clamp(x, max=0) * (1 - p) ** 2).sum()


def smooth_l1(t, x, mask):
    d = t - x
    v = torch.where(d.abs() < 1, 0.5 * d * d, d.abs())
    return (v * mask.unsqueeze(-1)).sum()


def iou(t, x, mask):
    th, tw = t[..., 0] + t[..., 1], t[..., 2] + t[..., 3]
    ph, pw = x[..., 0] + x[..., 1], x[..., 2] + x[..., 3]
    ih = torch.clamp(torch.minimum(t[..., 1], x[..., 1]) + torch.minimum(t[..., 0], x[..., 0]), min=0)
    iw = torch.clamp(torch.minimum(t[..., 3], x[..., 3]) + torch.minimum(t[..., 2], x[..., 2]), min=0)
    inter = ih * iw
    u = th * tw + ph * pw - inter
    io = inter / (u + 1e-12)
    return (-torch.log(io + 1e-12) * mask).sum()


def packed_loss(reg, cls, tgt, C, reg_type="l1"):
    """reg [N,>=5], cls [N,>=C], tgt [N,5+C] (float64 tensors, requires_grad on reg/cls)."""
    mask = (tgt[:, 5:5 + C].max(-1).values >= 1).to(tgt.dtype)
    lc = focal(tgt[:, 5:5 + C], cls[:, :C])
    d = tgt[:, 4] - torch.sigmoid(reg[:, 4])
    le = torch.where(d.abs() < 1, 0.5 * d * d, d.abs()).sum()
    if reg_type == "iou":
        lr = iou(tgt[:, :4], reg[:, :4], mask)
    else:
        lr = smooth_l1(tgt[:, :4], reg[:, :4], mask)
    return lc, lr, le


def centre_packed_loss(reg, cen, cls, tgt, C, reg_type="l1", cen_type="focal", reg_sigmoid=False):
    """FCOS/fcos_center.py:365-399 / fcos_center_v1.py:283-317 (oracle/fcos_ref.center_model_loss):
    reg [N,>=4] raw head (sigmoid'd first when reg_sigmoid), cen [N] logit, cls [N,>=C]."""
    mask = (tgt[:, 5:5 + C].max(-1).values >= 1).to(tgt.dtype)
    lc = focal(tgt[:, 5:5 + C], cls[:, :C])
    if cen_type == "focal":
        le = focal(tgt[:, 4], cen)
    else:
        d = tgt[:, 4] - torch.sigmoid(cen)
        le = torch.where(d.abs() < 1, 0.5 * d * d, d.abs()).sum()
    r = torch.sigmoid(reg[:, :4]) if reg_sigmoid else reg[:, :4]
    lr = iou(tgt[:, :4], r, mask) if reg_type == "iou" else smooth_l1(tgt[:, :4], r, mask)
    return lc, lr, le
