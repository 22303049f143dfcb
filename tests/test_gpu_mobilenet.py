"""MobileNetV2 backbone (tf.keras.applications.MobileNetV2 as FCOS/fcos.py:36-41, RetinaNet and the
CenterNet modules use it) on the GPU.

  * cvl_depthwise_fwd / dgrad / wgrad vs float64 torch (groups = C) on the same bf16 operands
    (bf16 outputs within 1e-2 rel-L2 ... 1 bf16 rounding; fp32 weight gradient 1e-4), stride 1
    "same" and stride 2 ZeroPadding2D((0,1),(0,1)) + valid, padded channel pitches, beta;
  * BN -> ReLU6 apply (relu = 2) and backward (mask 0 < bn(z) < 6 from z) vs float64 autograd;
  * FCOS on MobileNetV2 (every backbone_model but "resnet50" in fcos.py): forward, loss and every
    gradient vs the oracle restatement (oracle/model_ref.mobilenet_v2) with bf16 storage emulated,
    residual-branch BN gammas damped so the random-init graph is not chaotic; zero channel pads stay
    zero; a captured train step stays finite.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _pads(s):
    return (1, 1, 1, 1) if s == 1 else (0, 1, 0, 1)


@pytest.mark.parametrize("B,H,W,C,s", [(2, 16, 16, 32, 1), (2, 16, 16, 160, 2), (1, 9, 12, 64, 1), (2, 8, 8, 960, 1),
                                       (2, 64, 160, 128, 1),       # hourglass split-conv form (row walk)
                                       (3, 14, 10, 96, 2)])
def test_depthwise_fwd_dgrad_wgrad(B, H, W, C, s):
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(C + s)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    w = torch.randn(3, 3, C, 1, generator=g) * 0.3
    pt = pl = 1 if s == 1 else 0
    Ho, Wo = (H, W) if s == 1 else ((H - 2) // 2 + 1, (W - 2) // 2 + 1)
    y = torch.empty((B, Ho, Wo, C), dtype=torch.bfloat16, device="cuda")
    nn.depthwise_fwd(x.cuda(), w.cuda(), y, 3, s, pt, pl)
    xd = x.double().permute(0, 3, 1, 2).requires_grad_()
    wd = w.double().requires_grad_()
    ref = F.conv2d(F.pad(xd, _pads(s)), wd.permute(2, 3, 0, 1), None, s, groups=C)
    assert ref.shape[2:] == (Ho, Wo)
    assert rel(y.permute(0, 3, 1, 2), ref.detach()) < 4e-3
    dy = torch.randn(B, Ho, Wo, C, generator=g).to(torch.bfloat16)
    ref.backward(dy.double().permute(0, 3, 1, 2))
    dx = torch.full((B, H, W, C), 0.5, dtype=torch.bfloat16, device="cuda")
    nn.depthwise_dgrad(dy.cuda(), w.cuda(), dx, 3, s, pt, pl, beta=1.0)
    assert rel(dx.permute(0, 3, 1, 2), xd.grad + 0.5) < 4e-3
    dw = torch.full((3, 3, C, 1), 0.25, device="cuda")
    nn.depthwise_wgrad(x.cuda(), dy.cuda(), dw, 3, s, pt, pl, beta=2.0)
    assert rel(dw, wd.grad + 0.5) < 1e-4


def test_bn_relu6_apply_and_backward():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(9)
    B, H, W, C = 2, 10, 12, 64
    z = (torch.randn(B, H, W, C, generator=g) * 4 + 2).to(torch.bfloat16).cuda()
    gamma = (torch.rand(C, generator=g) * 2 + 0.5).cuda()
    beta = (torch.randn(C, generator=g) * 2).cuda()
    stats = nn.bn_acc(B, C, "cuda")
    nn.bn_stats(z, B, H * W, C, stats)
    mr = torch.empty((B, C, 2), device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nn.bn_finalize_grouped(stats, mr, rm, rv, B, C, H * W, 1, 1e-3, 0.999)
    y = torch.empty_like(z)
    nn.bn_apply(z, mr, gamma, beta, None, y, B, H * W, C, 2)
    zd = z.double().cpu().requires_grad_()
    m = zd.mean((1, 2), keepdim=True)
    v = ((zd - m) ** 2).mean((1, 2), keepdim=True)
    yr = torch.clamp((zd - m) / torch.sqrt(v + 1e-3) * gamma.double().cpu() + beta.double().cpu(), 0, 6)
    assert rel(y, yr.detach()) < 1e-2 and float(y.float().max()) <= 6.0
    assert (y.float() == 6.0).any() and (y.float() == 0.0).any()
    dy = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).cuda()
    (gz,) = torch.autograd.grad(yr, zd, dy.double().cpu())
    dz = torch.empty_like(z)
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    nn.bn_backward_relu6(dy, z, mr, gamma, beta, dz, dg, db, B, H * W, C)
    assert rel(dz, gz) < 1e-2


def _damp(net, factor):
    for k in net.store.offsets:
        if k.endswith("project_BN/gamma"):
            net.store.p(k).mul_(factor)


def test_fcos_mobilenetv2_graph_vs_oracle():
    from cvlite import ops_targets as ot
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, backbone_model="mobilenetv2", seed=3)
    assert type(net.backbone).__name__ == "MobileNetV2"
    assert type(FCOSNet(C, backbone_model="resnet101", seed=0).backbone).__name__ == "MobileNetV2"   # fcos.py:35-41
    _damp(net, 0.25)
    params = net.store.state_dict()
    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.uniform(-1, 1, size=(B, D, D, 3)).astype(np.float32))
    boxes = np.zeros((B, 4, 5), np.float32)
    boxes[:, :, :2] = rng.uniform(0.3, 0.7, (B, 4, 2))
    boxes[:, :, 2:4] = rng.uniform(0.1, 0.5, (B, 4, 2))
    boxes[:, :, 4] = rng.integers(0, C, (B, 4))
    nbox = np.full(B, 4, np.int32)
    dims = torch.full((B, 2), float(D), device="cuda")
    tg, _ = ot.fcos_assign(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), dims, (D, D), C)
    reg, cls = net.forward(x.cuda())
    P = reg.shape[1]
    d_reg = torch.zeros((B, P, 32), dtype=torch.bfloat16, device="cuda")
    d_cls = torch.zeros((B, P, net.cls_ld), dtype=torch.bfloat16, device="cuda")
    losses, _, _ = ot.fcos_loss(reg, cls, tg, C, grad_scale=1.0 / B, d_reg=d_reg, d_cls=d_cls)
    net.backward(d_reg, d_cls)
    torch.cuda.synchronize()
    # pads of the channel-padded maps / parameters stay exactly zero
    for k in net.store.offsets:
        if k.startswith("block_1_expand/") or k.startswith("expanded_conv_project/"):
            pass
    w = net.store.p("block_2_depthwise/depthwise_kernel")
    assert not w[:, :, 144:].any() and not net.store.g("block_2_depthwise/depthwise_kernel")[:, :, 144:].any()
    assert not net.store.g("expanded_conv_project/kernel")[..., 16:].any()
    tgc = tg.cpu()
    with model_ref.emulate_bf16():
        l16, g16, reg16, cls16 = model_ref.fcos_loss_and_grads(params, x, tgc, C, grad_scale=1.0 / B)
    l32, g32, reg32, cls32 = model_ref.fcos_loss_and_grads(params, x, tgc, C, grad_scale=1.0 / B)
    er, ec = rel(reg[..., :5].cpu(), reg16), rel(cls[..., :C].cpu(), cls16)
    print("reg %.4f cls %.4f | bf16-oracle vs fp32: %.4f %.4f" % (er, ec, rel(reg16, reg32), rel(cls16, cls32)))
    assert er < max(2e-2, 1.5 * rel(reg16, reg32)) and ec < max(2e-2, 1.5 * rel(cls16, cls32))
    assert rel(losses.double(), l16.double()) < 3e-2
    big = max(float(v.norm()) for v in g32.values())
    excess = []
    for k, gr in g32.items():
        if float(gr.norm()) < 1e-3 * big or k.endswith("_conv/bias"):
            continue
        e_gpu, e_emu = rel(net.store.g(k).cpu(), gr), rel(g16[k], gr)
        # per tensor within 2x the bf16-storage oracle's own divergence + 0.1, the bound the FCOS
        # whole-graph test uses (chaotic random-init tensors reach rel-L2 ~0.7 in the oracle itself)
        excess.append((e_gpu - (2.0 * e_emu + 0.1), e_gpu, e_emu, k))
    excess.sort(reverse=True)
    print("worst (excess, gpu, bf16-oracle, tensor):", excess[:4])
    assert excess[0][0] <= 0, excess[:4]
    n_bb = sum(1 for e in excess if e[3].startswith(("block_", "expanded_conv_", "Conv1", "bn_Conv1", "Conv_1")))
    print("backbone tensors compared:", n_bb)
    assert n_bb > 40


def test_fcos_mobilenetv2_train_step():
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    net = FCOSNet(20, backbone_model="mobilenetv2", seed=0)
    tr = FCOSTrainer(net, 2, (256, 256))
    imgs, boxes, nbox = synthetic_batch(2, 256, 256, 20, seed=5)
    w0 = net.store.flat.clone()
    for _ in range(2):
        tr.load_batch(imgs, boxes, nbox)
        losses = tr.step()
    torch.cuda.synchronize()
    assert torch.isfinite(losses).all() and torch.isfinite(net.store.flat).all()
    assert not torch.equal(w0, net.store.flat)
