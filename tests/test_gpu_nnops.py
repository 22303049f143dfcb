"""GPU parity of the memory-bound ops (BN fwd/bwd with per-image stats, max-pool, FPN upsample,
ReLU backward, bias grad, clip+SGD, LR schedule) against torch fp64 references."""
import math

import numpy as np

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def bfr(t):
    return t.to(BF).to(torch.float64)


@pytest.mark.parametrize("B,HW,C,relu,res", [(2, 64, 64, True, False), (3, 16, 256, False, True),
                                             (1, 256, 32, True, True), (2, 1000, 64, True, False),
                                             (1, 300, 2048, True, True), (2, 4096, 256, True, False)])
def test_bn_forward_backward(B, HW, C, relu, res):
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B * 100 + C)
    z = bfr(torch.randn(B, HW, C, generator=g, dtype=torch.float64) * 2 + 0.5)
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64)
    r = bfr(torch.randn(B, HW, C, generator=g, dtype=torch.float64)) if res else None
    eps = 1.001e-5
    stats = nn.bn_acc_encode(torch.stack([z.sum(1), (z * z).sum(1)], -1)).cuda()
    mr = torch.empty((B, C, 2), dtype=torch.float32, device="cuda")
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    nn.bn_finalize(stats, mr, rm, rv, B, C, HW, eps, 0.99)
    y = torch.empty((B, HW, C), dtype=BF, device="cuda")
    zg = z.to(BF).cuda()
    nn.bn_apply(zg, mr, gamma.float().cuda(), beta.float().cuda(), r.to(BF).cuda() if res else None, y, B, HW,
                C, relu)
    zz = z.clone().requires_grad_(True)
    gg = gamma.clone().requires_grad_(True)
    bb = beta.clone().requires_grad_(True)
    m = zz.mean(1, keepdim=True)
    v = ((zz - m) ** 2).mean(1, keepdim=True)
    out = (zz - m) / torch.sqrt(v + eps) * gg + bb
    if res:
        out = out + r
    if relu:
        out = F.relu(out)
    torch.testing.assert_close(y.double().cpu(), out.detach(), rtol=1e-2, atol=2e-2)
    # running stats: sequential EMA over images, unbiased variance
    erm, erv = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    for b in range(B):
        erm = erm * 0.99 + m[b, 0] * 0.01
        erv = erv * 0.99 + v[b, 0] * HW / (HW - 1) * 0.01
    torch.testing.assert_close(rm.double().cpu(), erm.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double().cpu(), erv.detach(), rtol=1e-5, atol=1e-6)
    # the fused finalize+apply launch is bit-identical to the two-launch path
    mr2 = torch.empty_like(mr)
    rm2, rv2 = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y2 = torch.empty_like(y)
    nn.bn_finalize_apply(stats, mr2, rm2, rv2, zg, gamma.float().cuda(), beta.float().cuda(),
                         r.to(BF).cuda() if res else None, y2, B, HW, C, relu, eps, 0.99)
    assert torch.equal(mr2, mr) and torch.equal(rm2, rm) and torch.equal(rv2, rv)
    assert torch.equal(y2.view(torch.int16), y.view(torch.int16))
    # backward
    dy = bfr(torch.randn(B, HW, C, generator=g, dtype=torch.float64))
    out.backward(dy)
    dz = torch.empty_like(zg)
    gout = torch.empty_like(zg)
    dgam = torch.zeros(C, device="cuda")
    dbet = torch.zeros(C, device="cuda")
    cdb = torch.full((C,), 7.0, device="cuda")
    nn.bn_backward(dy.to(BF).cuda(), y if relu else None, zg, mr, gamma.float().cuda(), dz, gout, dgam, dbet,
                   B, HW, C, conv_dbias=cdb)
    scale = zz.grad.abs().max().item()
    torch.testing.assert_close(dz.double().cpu(), zz.grad, rtol=2e-2, atol=2e-2 * scale)
    # gradient of the preceding conv's bias: exactly 0 behind training-mode BN (fp64 autograd agrees)
    assert torch.count_nonzero(cdb).item() == 0
    torch.testing.assert_close(cdb.double().cpu(), zz.grad.sum((0, 1)), rtol=0, atol=1e-8 * scale * B * HW)
    if relu:
        torch.testing.assert_close(gout.double().cpu(), dy * (y.double().cpu() > 0))
    torch.testing.assert_close(dgam.double().cpu(), gg.grad, rtol=2e-2, atol=2e-2 * gg.grad.abs().max().item())
    torch.testing.assert_close(dbet.double().cpu(), bb.grad, rtol=2e-2, atol=2e-2 * bb.grad.abs().max().item())
    if relu and not res:
        # the non-residual form rebuilds the ReLU mask from z: bit-identical to reading y
        dz2, dgam2, dbet2 = torch.empty_like(zg), torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        cdb2 = torch.full((C,), 7.0, device="cuda")
        nn.bn_backward_relu(dy.to(BF).cuda(), zg, mr, gamma.float().cuda(), beta.float().cuda(), dz2, dgam2, dbet2,
                            B, HW, C, conv_dbias=cdb2)
        assert torch.equal(dz2.view(torch.int16), dz.view(torch.int16))
        assert torch.equal(dgam2, dgam) and torch.equal(dbet2, dbet) and torch.count_nonzero(cdb2).item() == 0


@pytest.mark.parametrize("B,HW,C", [(2, 64, 256), (3, 256, 2048), (1, 4096, 512)])
def test_bn_finalize_apply_bnres_bit_identical(B, HW, C):
    """cvl_bn_finalize_apply_bnres (projection shortcut's BN formed inside conv3's BN launch) equals
    the two-launch form bit for bit: shortcut finalize_apply (no ReLU) stored as bf16, then conv3's
    finalize_apply with it as the residual -- y, both (mean, rstd) and both running statistics."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B * 7 + C)
    dev = "cuda"
    z = bfr(torch.randn(B, HW, C, generator=g, dtype=torch.float64) * 2 + 0.5)
    zs = bfr(torch.randn(B, HW, C, generator=g, dtype=torch.float64) * 3 - 0.2)
    ga, be = (torch.rand(C, generator=g) + 0.5).cuda(), torch.randn(C, generator=g).cuda()
    gs, bs = (torch.rand(C, generator=g) + 0.5).cuda(), torch.randn(C, generator=g).cuda()
    st = nn.bn_acc_encode(torch.stack([z.sum(1), (z * z).sum(1)], -1)).cuda()
    sts = nn.bn_acc_encode(torch.stack([zs.sum(1), (zs * zs).sum(1)], -1)).cuda()
    zg, zsg = z.to(BF).cuda(), zs.to(BF).cuda()
    outs = []
    for fused in (False, True):
        mr, mrs = torch.empty((B, C, 2), device=dev), torch.empty((B, C, 2), device=dev)
        rm, rv, rms, rvs = (torch.full((C,), v, device=dev) for v in (0.1, 1.1, -0.2, 0.9))
        y = torch.empty_like(zg)
        if fused:
            nn.bn_finalize_apply_bnres(st.clone(), mr, rm, rv, zg, ga, be, sts.clone(), mrs, rms, rvs, zsg, gs, bs,
                                       1e-3, 0.9, y, B, HW, C, 1, 1.001e-5, 0.99)
        else:
            s = torch.empty_like(zg)
            nn.bn_finalize_apply(sts.clone(), mrs, rms, rvs, zsg, gs, bs, None, s, B, HW, C, 0, 1e-3, 0.9)
            nn.bn_finalize_apply(st.clone(), mr, rm, rv, zg, ga, be, s, y, B, HW, C, 1, 1.001e-5, 0.99)
        outs.append((y.view(torch.int16), mr, mrs, rm, rv, rms, rvs))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_maxpool_and_upsample():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(11)
    B, H, W, C = 2, 14, 10, 64
    x = bfr(torch.relu(torch.randn(B, H, W, C, generator=g, dtype=torch.float64)))
    x[0, :3, :3, :8] = 0.0                         # ties with the zero padding
    xx = x.clone().requires_grad_(True)
    ref = F.max_pool2d(F.pad(xx.permute(0, 3, 1, 2), (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1)
    Ho, Wo = ref.shape[1], ref.shape[2]
    y = torch.empty((B, Ho, Wo, C), dtype=BF, device="cuda")
    arg = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device="cuda")
    nn.maxpool3x3s2(x.to(BF).cuda(), y, arg)
    torch.testing.assert_close(y.double().cpu(), ref.detach())
    dy = bfr(torch.randn(B, Ho, Wo, C, generator=g, dtype=torch.float64))
    ref.backward(dy)
    dx = torch.empty((B, H, W, C), dtype=BF, device="cuda")
    nn.maxpool3x3s2_backward(dy.to(BF).cuda(), arg, dx)
    torch.testing.assert_close(dx.double().cpu(), xx.grad, rtol=1e-2, atol=1e-2)
    # upsample-add and its backward
    a = bfr(torch.randn(B, 8, 6, C, generator=g, dtype=torch.float64))
    b = bfr(torch.randn(B, 4, 3, C, generator=g, dtype=torch.float64))
    o = torch.empty((B, 8, 6, C), dtype=BF, device="cuda")
    nn.upsample2x_add(a.to(BF).cuda(), b.to(BF).cuda(), o, B, 8, 6, C)
    up = b.repeat_interleave(2, 1).repeat_interleave(2, 2)
    torch.testing.assert_close(o.double().cpu(), a + up, rtol=1e-2, atol=1e-2)
    do = bfr(torch.randn(B, 8, 6, C, generator=g, dtype=torch.float64))
    db = b.to(BF).cuda()
    nn.upsample2x_backward(do.to(BF).cuda(), db, B, 8, 6, C, beta=1.0)
    exp = b + do.reshape(B, 4, 2, 3, 2, C).sum((2, 4))
    torch.testing.assert_close(db.double().cpu(), exp, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("B,H,W", [(2, 256, 256), (3, 37, 70)])
def test_stem_pool_tiled_forms_match_generic(B, H, W):
    """The 64-channel tiled kernels of the stem pool (bn_relu_maxpool64, maxpool_bwd64: one LDS tile
    of relu(BN(z)) / of the windows' dy + argmax per workgroup) are bit-identical to the generic
    per-output kernels, which serve any other C: the first 64 channels of a 128-channel run."""
    from cvlite import ops_nn as nn
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(H + W)
    z = (torch.randn(B, H, W, 128, generator=g) * 2.0).to(BF).to(dev)
    mr = torch.stack([torch.randn(B, 128, generator=g) * 0.3, torch.rand(B, 128, generator=g) + 0.5], -1).float().to(dev)
    gamma = (torch.rand(128, generator=g) + 0.5).to(dev)
    beta = (torch.randn(128, generator=g) * 0.5).to(dev)
    Ho, Wo = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    p128 = torch.empty((B, Ho, Wo, 128), dtype=BF, device=dev)
    a128 = torch.empty((B, Ho, Wo, 128), dtype=torch.uint8, device=dev)
    nn.bn_relu_maxpool3x3s2(z, mr, gamma, beta, p128, a128)
    z64 = z[..., :64].contiguous()
    mr64 = mr[:, :64].contiguous()
    p64 = torch.empty((B, Ho, Wo, 64), dtype=BF, device=dev)
    a64 = torch.empty((B, Ho, Wo, 64), dtype=torch.uint8, device=dev)
    nn.bn_relu_maxpool3x3s2(z64, mr64, gamma[:64].contiguous(), beta[:64].contiguous(), p64, a64)
    assert torch.equal(p64.view(torch.int16), p128[..., :64].contiguous().view(torch.int16))
    assert torch.equal(a64, a128[..., :64].contiguous())
    dy = (torch.randn(B, Ho, Wo, 128, generator=g)).to(BF).to(dev)
    dx128 = torch.empty((B, H, W, 128), dtype=BF, device=dev)
    nn.maxpool3x3s2_backward(dy, a128, dx128)
    dx64 = torch.empty((B, H, W, 64), dtype=BF, device=dev)
    nn.maxpool3x3s2_backward(dy[..., :64].contiguous(), a64, dx64)
    assert torch.equal(dx64.view(torch.int16), dx128[..., :64].contiguous().view(torch.int16))


def test_relu_bwd_bias_grad_sgd_lr():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(5)
    dy = bfr(torch.randn(4096, generator=g, dtype=torch.float64))
    y = bfr(torch.randn(4096, generator=g, dtype=torch.float64))
    dx = torch.empty(4096, dtype=BF, device="cuda")
    nn.relu_backward(dy.to(BF).cuda(), y.to(BF).cuda(), dx)
    torch.testing.assert_close(dx.double().cpu(), dy * (y > 0))
    # bias grad over a segment of an image-major [B, P, ld] buffer
    B, P, ld = 3, 50, 32
    t = bfr(torch.randn(B, P, ld, generator=g, dtype=torch.float64))
    db = torch.ones(20, device="cuda")
    nn.bias_grad(t.to(BF).cuda(), ld, 0, 20, 10, P, 16, B, db, beta=1.0)
    torch.testing.assert_close(db.double().cpu(), 1 + t[:, 10:26, :20].sum((0, 1)), rtol=1e-5, atol=1e-4)
    for (B, P, ld, coff, ncol, base, HW) in ((16, 5456, 32, 0, 5, 4096, 1024), (16, 5456, 256, 0, 256, 0, 4096),
                                             (2, 777, 64, 8, 40, 3, 700)):
        t = bfr(torch.randn(B, P, ld, generator=g, dtype=torch.float64))
        db = torch.zeros(ncol, device="cuda")
        nn.bias_grad(t.to(BF).cuda(), ld, coff, ncol, base, P, HW, B, db)
        exp = t[:, base:base + HW, coff:coff + ncol].sum((0, 1))
        torch.testing.assert_close(db.double().cpu(), exp, rtol=1e-5, atol=1e-3)
    # batched form: FCOS heads (5 levels x 2 heads at 512 / bs 16), a RetinaNet 720-column head,
    # an FPN-style level of a packed [rows, 256] buffer, a beta-accumulating item; one launch pair
    B, P = 16, 5456
    d_cls = bfr(torch.randn(B, P, 32, generator=g, dtype=torch.float64))
    d_ret = bfr(torch.randn(2, 300, 736, generator=g, dtype=torch.float64))
    fpn = bfr(torch.randn(B * 100 + 37, 256, generator=g, dtype=torch.float64))
    dc, dr, df = d_cls.to(BF).cuda(), d_ret.to(BF).cuda(), fpn.to(BF).cuda()
    items, exps = [], []
    off = 0
    for s in (64, 32, 16, 8, 4):
        for ncol in (20, 5):
            db = torch.zeros(ncol, device="cuda")
            items.append((dc, 32, 0, ncol, off, P, s * s, B, db, 0.0))
            exps.append((db, d_cls[:, off:off + s * s, :ncol].sum((0, 1))))
        off += s * s
    db = torch.zeros(720, device="cuda")
    items.append((dr, 736, 0, 720, 17, 300, 250, 2, db, 0.0))
    exps.append((db, d_ret[:, 17:267, :720].sum((0, 1))))
    # the widest item (2048 columns: one row per pass), single-row images, a partly filled
    # column-group tile (65 groups of 8 -> 128 threads per row)
    wide = bfr(torch.randn(2, 40, 2048, generator=g, dtype=torch.float64))
    db = torch.zeros(2048, device="cuda")
    items.append((wide.to(BF).cuda(), 2048, 0, 2048, 3, 40, 33, 2, db, 0.0))
    exps.append((db, wide[:, 3:36].sum((0, 1))))
    one = bfr(torch.randn(3, 2, 528, generator=g, dtype=torch.float64))
    db = torch.zeros(520, device="cuda")
    items.append((one.to(BF).cuda(), 528, 8, 520, 1, 2, 1, 3, db, 0.0))
    exps.append((db, one[:, 1, 8:528].sum(0)))
    db = torch.full((256,), 2.0, device="cuda")
    items.append((df, 256, 0, 256, 37, 100, 100, B, db, 0.5))
    exps.append((db, 1.0 + fpn[37:].reshape(B, 100, 256).sum((0, 1))))
    nn.bias_grad_multi(items)
    for db, exp in exps:
        torch.testing.assert_close(db.double().cpu(), exp, rtol=1e-5, atol=2e-3)
    # deterministic: a second launch gives the same bits
    first = [db.clone() for db, _ in exps[:-1]]
    nn.bias_grad_multi(items[:-1])
    for a, (db, _) in zip(first, exps[:-1]):
        assert torch.equal(a, db)
    # clip + SGD (Keras form), lr from device memory
    n = 100003
    w = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g) * 3
    v = torch.randn(n, generator=g) * 0.1
    lr = 5e-4
    wd, gd, vd = w.cuda(), gr.cuda(), v.cuda()
    lr_dev = torch.tensor([lr], device="cuda")
    nn.sgd_clip_update(wd, gd, vd, lr_dev, 0.9, 1.0 / 16, 1.0)
    gg = gr.double() / 16
    norm = gg.norm().item()
    gg = gg * (1.0 / max(norm, 1.0))
    ev = 0.9 * v.double() - lr * gg
    torch.testing.assert_close(vd.double().cpu(), ev, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(wd.double().cpu(), w.double() + ev, rtol=1e-5, atol=1e-6)
    # lr schedule (train_fcos.py:108-110)
    step = torch.tensor([0], dtype=torch.int32, device="cuda")
    lrd = torch.zeros(1, device="cuda")
    for s in (0, 999, 1000, 2500, 60000):
        step.fill_(s)
        nn.lr_schedule(step, lrd, 5e-4, 1e-5, 0.9, 1000)
        exp = max(5e-4 * math.pow(0.9, int(s / 1000)), 1e-5)
        assert abs(lrd.item() - np.float32(exp)) == 0, (s, lrd.item(), exp)
        assert step.item() == s + 1


def test_pack_multi_matches_single():
    """cvl_pack_conv_weights_multi (one launch for every conv) == per-conv cvl_pack_conv_weights."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(11)
    specs = [(3, 256, 256, 256, 256, 256, 256), (1, 1024, 256, 1024, 256, 1024, 256), (3, 256, 20, 256, 32, 256, 32),
             (3, 256, 5, 256, 32, 256, 32), (1, 147, 64, 160, 64, 0, 0), (3, 2048, 256, 2048, 256, 2048, 256),
             (7, 96, 40, 96, 64, 96, 64)]
    entries, ref = [], []
    for (k, cin, cout, cin_k, npad, cin_pad, cout_pad) in specs:
        w = torch.randn(k, k, cin, cout, generator=g).cuda()
        khw = k * k
        wf = torch.full((npad, khw * cin_k), 7.0, dtype=BF, device="cuda")
        wd = torch.full((cin_pad, khw * cout_pad), 7.0, dtype=BF, device="cuda") if cin_pad else None
        entries.append((w, khw, cin, cout, cin_k, npad, wf, cin_pad, cout_pad, wd))
        rf = torch.empty_like(wf)
        rd = torch.empty_like(wd) if wd is not None else None
        nn.pack_conv_weights(w, k, k, cin, cout, cin_k, npad, rf, cin_pad, cout_pad, rd)
        ref.append((rf, rd))
    plan = nn.PackPlan(entries, "cuda")
    plan.run()
    torch.cuda.synchronize()
    for e, (rf, rd) in zip(entries, ref):
        assert torch.equal(e[6], rf)
        if rd is not None:
            assert torch.equal(e[9], rd)


@pytest.mark.parametrize("B,H,W,stride,Kp,C,K", [(2, 37, 29, 2, 160, 3, 7), (1, 64, 300, 2, 152, 3, 7),
                                                 (3, 20, 18, 1, 150, 3, 7), (2, 21, 19, 2, 80, 8, 3)])
def test_im2col_matches_unfold(B, H, W, stride, Kp, C, K):
    """ResNet/hourglass stem im2col (7x7, C=3, TF-same pads) vs torch unfold: the LDS-tiled stem
    kernel (several 64-pixel segments per row at W=300), the 16-byte generic one (C=8) and the
    scalar one (Kp % 8 != 0).  Exact (bf16 rounding of the same fp32 values)."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(H * W)
    x = torch.randn(B, H, W, C, generator=g)
    Ho, Wo = -(-H // stride), -(-W // stride)
    ph = max((Ho - 1) * stride + K - H, 0)
    pw = max((Wo - 1) * stride + K - W, 0)
    pt, pl = ph // 2, pw // 2
    out = torch.full((B * Ho * Wo, Kp), 7.0, dtype=BF, device="cuda")
    nn.im2col(x.cuda(), K, K, stride, pt, pl, Ho, Wo, Kp, out)
    xp = F.pad(x.permute(0, 3, 1, 2), (pl, pw - pl, pt, ph - pt))
    cols = F.unfold(xp, K, stride=stride)                    # [B, C*K*K (c, r, s), Ho*Wo]
    cols = cols.view(B, C, K * K, Ho * Wo).permute(0, 3, 2, 1).reshape(B * Ho * Wo, K * K * C)
    ref = torch.zeros(B * Ho * Wo, Kp)
    ref[:, :K * K * C] = cols
    assert torch.equal(out.cpu().view(torch.int16), ref.to(BF).view(torch.int16))


@pytest.mark.parametrize("B,H,Cin,Cout,k,expect_fused", [
    (2, 128, 64, 64, 3, True),       # conv2_x 3x3 data gradient -> conv2_x conv1 BN (L64 kernel)
    (8, 64, 512, 128, 1, True),      # conv3_x conv3 1x1 data gradient -> conv2 BN (persistent 1x1 kernel)
    (16, 128, 256, 64, 1, True),     # conv2_x conv3 1x1 data gradient at bs 16 (persistent, 4 tiles per workgroup)
    (2, 16, 2048, 512, 1, True),     # conv5_x: one tile per image (persistent 1x1 kernel)
    (2, 12, 256, 64, 1, False),      # H*W % 256 != 0: no per-image tiles -> plain path
])
def test_dgrad_fused_bn_backward_first_pass(B, H, Cin, Cout, k, expect_fused):
    """cvl_conv_igemm_dgrad_bnsum + cvl_bn_backward_relu_sums (the first BN-backward pass formed in
    the data-gradient epilogue) against the plain data gradient + two-pass cvl_bn_backward_relu on
    the same operands: dX bit-identical, first-pass sums within fp32 summation order, dz / dgamma /
    dbeta within one bf16 rounding; the unfusable launch reports fused=False and leaves sums 0."""
    from cvlite import ops_nn as nn
    from cvlite.layers import Conv, ParamStore
    W = H
    C = Cout                     # dgrad output channels = the conv's input channels = the BN's channels
    dev = torch.device("cuda")
    st = ParamStore()
    conv = Conv(st, "c", k, C, Cin, 1, "same", bias=False)     # forward C -> Cin; its dgrad yields dC
    st.finalize(dev, seed=3)
    conv.pack()
    g = torch.Generator(device="cpu").manual_seed(B + H + Cin)
    dy_next = (torch.randn(B, H, W, Cin, generator=g) * 0.5).to(BF).to(dev)
    z = (torch.randn(B, H, W, C, generator=g) * 1.5 + 0.2).to(BF).to(dev)
    mr = torch.empty((B, C, 2), dtype=torch.float32, device=dev)
    zf = z.double().view(B, H * W, C)
    mr[..., 0] = zf.mean(1).float()
    mr[..., 1] = torch.rsqrt(zf.var(1, unbiased=False) + 1e-3).float()
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = torch.randn(C, generator=g).to(dev) * 0.3
    d = conv.dgrad_desc(B, [nn.seg(H, W, H, W, conv.wd)], ld_dst=C)
    # fused
    dx_f = torch.empty((B, H, W, C), dtype=BF, device=dev)
    sums = nn.bn_acc(B, C, dev)
    fused = nn.conv_igemm_dgrad_bnsum(d, dy_next, dx_f, z, mr, gamma, beta, sums)
    assert fused == expect_fused
    # plain
    dx_p = torch.empty_like(dx_f)
    nn.conv_igemm(d, dy_next, dx_p)
    assert torch.equal(dx_f, dx_p)
    if not expect_fused:
        assert float(sums.abs().max()) == 0.0
        return
    # reference first-pass sums (fp64 on the same bf16 values)
    xh = (z.float() - mr[..., 0].view(B, 1, 1, C)) * mr[..., 1].view(B, 1, 1, C)
    a = gamma * xh + beta
    gm = torch.where(a > 0, dx_p.float(), torch.zeros_like(a)).double()
    ref = torch.stack([gm.sum((1, 2)), (gm * xh.double()).sum((1, 2))], -1)
    torch.testing.assert_close(nn.bn_acc_value(sums), ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))
    HW = H * W
    dz_f, dz_p = torch.empty_like(z), torch.empty_like(z)
    dg_f, db_f = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dg_p, db_p = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    nn.bn_backward_relu_sums(dx_f, z, mr, gamma, beta, sums, dz_f, dg_f, db_f, B, HW, C)
    nn.bn_backward_relu(dx_p, z, mr, gamma, beta, dz_p, dg_p, db_p, B, HW, C)
    torch.testing.assert_close(dz_f.float(), dz_p.float(), rtol=1e-2, atol=1e-2 * float(dz_p.float().abs().max()))
    torch.testing.assert_close(dg_f, dg_p, rtol=1e-5, atol=1e-5 * float(dg_p.abs().max()))
    torch.testing.assert_close(db_f, db_p, rtol=1e-5, atol=1e-5 * float(db_p.abs().max()))


@pytest.mark.parametrize("B,H,Cin,Cout", [
    (16, 128, 64, 256),      # conv2_x: the next block's conv1 (256 -> 64) data gradient, 4 tiles per workgroup
    (8, 32, 256, 1024),      # conv4_x
    (4, 16, 512, 2048),      # conv5_x: one tile per image
])
def test_dgrad_fused_bn_backward_residual(B, H, Cin, Cout, dispatch):
    """cvl_conv_igemm_dgrad_bnsum_res + cvl_bn_backward_res_sums (a bottleneck's conv3 BN, whose dy the
    next block's conv1 data gradient completes by accumulating onto the shortcut gradient) against the
    plain accumulating data gradient + two-pass cvl_bn_backward with the y mask: dX bit-identical,
    first-pass sums within fp32 summation order, dz / g_out / dgamma / dbeta as the two-pass form."""
    from cvlite import ops_nn as nn
    from cvlite.layers import Conv, ParamStore
    dispatch("bnsum_res_min_hw=0")     # every map size (production floor: 256 px, i.e. conv5_x's 16x16 at 512)
    W = H
    C = Cout                     # block width: the BN3 channels = the next conv1's input channels
    dev = torch.device("cuda")
    st = ParamStore()
    conv = Conv(st, "c1", 1, C, Cin, 1, "same", bias=False)     # next block's conv1: C -> Cin
    st.finalize(dev, seed=5)
    conv.pack()
    g = torch.Generator(device="cpu").manual_seed(B + H + Cin)
    dy_next = (torch.randn(B, H, W, Cin, generator=g) * 0.5).to(BF).to(dev)
    old = (torch.randn(B, H, W, C, generator=g) * 0.5).to(BF).to(dev)      # the shortcut's gradient
    z = (torch.randn(B, H, W, C, generator=g) * 1.5 + 0.2).to(BF).to(dev)
    y = torch.relu(torch.randn(B, H, W, C, generator=g)).to(BF).to(dev)   # block output (zeros = masked)
    mr = torch.empty((B, C, 2), dtype=torch.float32, device=dev)
    zf = z.double().view(B, H * W, C)
    mr[..., 0] = zf.mean(1).float()
    mr[..., 1] = torch.rsqrt(zf.var(1, unbiased=False) + 1e-3).float()
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = torch.randn(C, generator=g).to(dev) * 0.3
    d = conv.dgrad_desc(B, [nn.seg(H, W, H, W, conv.wd)], ld_dst=C, beta=1.0)
    dx_f = old.clone()
    sums = nn.bn_acc(B, C, dev)
    assert nn.conv_igemm_dgrad_bnsum_res(d, dy_next, dx_f, y, z, mr, gamma, beta, sums)
    dx_p = old.clone()
    nn.conv_igemm(d, dy_next, dx_p)
    assert torch.equal(dx_f, dx_p)
    xh = (z.float() - mr[..., 0].view(B, 1, 1, C)) * mr[..., 1].view(B, 1, 1, C)
    gm = torch.where(y.float() > 0, dx_p.float(), torch.zeros_like(xh)).double()
    ref = torch.stack([gm.sum((1, 2)), (gm * xh.double()).sum((1, 2))], -1)
    torch.testing.assert_close(nn.bn_acc_value(sums), ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))
    HW = H * W
    dz_f, dz_p = torch.empty_like(z), torch.empty_like(z)
    go_f, go_p = torch.empty_like(z), torch.empty_like(z)
    dg_f, db_f = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dg_p, db_p = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    nn.bn_backward_res_sums(dx_f, y, z, mr, gamma, sums, dz_f, go_f, dg_f, db_f, B, HW, C)
    nn.bn_backward(dx_p, y, z, mr, gamma, dz_p, go_p, dg_p, db_p, B, HW, C)
    assert torch.equal(go_f, go_p)
    torch.testing.assert_close(dz_f.float(), dz_p.float(), rtol=1e-2, atol=1e-2 * float(dz_p.float().abs().max()))
    torch.testing.assert_close(dg_f, dg_p, rtol=1e-5, atol=1e-5 * float(dg_p.abs().max()))
    torch.testing.assert_close(db_f, db_p, rtol=1e-5, atol=1e-5 * float(db_p.abs().max()))
    if H * W < 4096:             # under a raised floor (round 5's 4096): the plain path, sums untouched
        dispatch("bnsum_res_min_hw=4096")
        sums2 = torch.zeros_like(sums)
        dx_2 = old.clone()
        assert not nn.conv_igemm_dgrad_bnsum_res(d, dy_next, dx_2, y, z, mr, gamma, beta, sums2)
        assert torch.equal(dx_2, dx_p) and float(sums2.abs().max()) == 0.0


@pytest.mark.parametrize("B,H,W", [(2, 256, 256), (3, 17, 23)])
def test_bn_relu_maxpool_matches_apply_then_pool(B, H, W):
    """cvl_bn_relu_maxpool3x3s2 (the stem's BN -> ReLU -> pad 1 -> max-pool 3x3/2 from z) equals
    cvl_bn_apply (ReLU) + cvl_maxpool3x3s2 on the same operands, pooled values and argmax bit-exact
    (zero padding ties and all-masked windows included)."""
    from cvlite import ops_nn as nn
    C = 64
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(B * H + W)
    z = (torch.randn(B, H, W, C, generator=g) * 2.0).to(BF).to(dev)
    mr = torch.stack([torch.randn(B, C, generator=g) * 0.3, torch.rand(B, C, generator=g) + 0.5], -1).float().to(dev)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.randn(C, generator=g) * 0.5).to(dev)
    Ho, Wo = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    y = torch.empty_like(z)
    nn.bn_apply(z, mr, gamma, beta, None, y, B, H * W, C, 1)
    p_ref = torch.empty((B, Ho, Wo, C), dtype=BF, device=dev)
    a_ref = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device=dev)
    nn.maxpool3x3s2(y, p_ref, a_ref)
    p = torch.empty_like(p_ref)
    a = torch.empty_like(a_ref)
    nn.bn_relu_maxpool3x3s2(z, mr, gamma, beta, p, a)
    assert torch.equal(p.view(torch.int16), p_ref.view(torch.int16))
    assert torch.equal(a, a_ref)


@pytest.mark.parametrize("B,H,W", [(2, 256, 256), (3, 17, 23)])
def test_maxpool_backward_bn_relu_fused(B, H, W):
    """cvl_maxpool3x3s2_backward_bn_relu (the stem's pool1 -> conv1_relu -> conv1_bn backward with the
    BN first pass inside the pool kernel) vs cvl_maxpool3x3s2_backward + cvl_bn_backward_relu: the
    pool gradient dy bit-exact, dz / dgamma / dbeta equal up to the order of the first-pass sums
    (fp32 partials over pool tiles instead of row chunks), conv_dbias zeroed; run to run bit-identical."""
    from cvlite import ops_nn as nn
    C = 64
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(B * H + W + 1)
    z = (torch.randn(B, H, W, C, generator=g) * 2.0).to(BF).to(dev)
    mr = torch.stack([torch.randn(B, C, generator=g) * 0.3, torch.rand(B, C, generator=g) + 0.5], -1).float().to(dev)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.randn(C, generator=g) * 0.5).to(dev)
    Ho, Wo = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    p = torch.empty((B, Ho, Wo, C), dtype=BF, device=dev)
    a = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device=dev)
    nn.bn_relu_maxpool3x3s2(z, mr, gamma, beta, p, a)
    dp = torch.randn((B, Ho, Wo, C), generator=g).to(BF).to(dev)
    dy_r, dz_r = torch.empty_like(z), torch.empty_like(z)
    dg_r, db_r = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    nn.maxpool3x3s2_backward(dp, a, dy_r)
    nn.bn_backward_relu(dy_r, z, mr, gamma, beta, dz_r, dg_r, db_r, B, H * W, C)
    outs = []
    for _ in range(2):
        dy, dz = torch.full_like(z, 7.0), torch.full_like(z, 7.0)
        dg, db, cb = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.full((C,), 3.0, device=dev)
        nn.maxpool3x3s2_backward_bn_relu(dp, a, z, mr, gamma, beta, dy, dz, dg, db, conv_dbias=cb)
        outs.append((dy, dz, dg, db, cb))
    dy, dz, dg, db, cb = outs[0]
    assert torch.equal(dy.view(torch.int16), dy_r.view(torch.int16))
    for x0, x1 in zip(outs[0], outs[1]):
        assert torch.equal(x0, x1)
    assert float(cb.abs().max()) == 0.0
    torch.testing.assert_close(dg, dg_r, rtol=1e-4, atol=1e-4 * float(dg_r.abs().max()))
    torch.testing.assert_close(db, db_r, rtol=1e-4, atol=1e-4 * float(db_r.abs().max()))
    d = (dz.float() - dz_r.float()).abs()
    assert float(d.max()) <= 2 ** -6 * float(dz_r.float().abs().max()), float(d.max())
    assert float((d > 0).float().mean()) < 0.02
