"""CenterNet hourglass training path on the GPU (CenterNet/tf_centernet_hourglass.py:87-564) vs the
torch-CPU restatement (oracle/centernet_model_ref.py) and torch fp64 references of each kernel.

Kernel tolerances: max-pool / argmax routing exact; bilinear up-sample within 1 bf16 ulp of the
fp32 reference on the same bf16 operands; fold/unfold 1e-6; grouped BN statistics and backward
vs fp64 autograd on the same bf16 inputs (bf16 output rounding, 1e-2 rel-L2); Adam 1e-6; loss 1e-5
and its bf16 gradient within bf16 rounding.  Whole graph: forward / loss / every gradient tensor vs
the bf16-storage oracle, rel-L2 <= 3e-2 (forward) and <= 0.1 over all gradients."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def bf(x):
    return x.to(torch.bfloat16)


def test_maxpool2x2_fwd_bwd():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(0)
    for (B, H, W, C) in [(2, 16, 16, 64), (3, 8, 12, 256), (1, 7, 9, 8)]:
        x = bf(torch.randn(B, H, W, C, generator=g)).cuda()
        x[0, :2, :2, :8] = 0            # ties: first maximum in window order takes the gradient
        Ho, Wo = (H + 1) // 2, (W + 1) // 2
        y = torch.empty((B, Ho, Wo, C), dtype=torch.bfloat16, device="cuda")
        arg = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device="cuda")
        nn.maxpool2x2(x, y, arg)
        ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 2, 2, ceil_mode=True).permute(0, 2, 3, 1)
        assert torch.equal(y.float(), ref)
        dy = bf(torch.randn(B, Ho, Wo, C, generator=g)).cuda()
        dx = torch.empty_like(x)
        nn.maxpool2x2_backward(dy, arg, dx)
        # reference routing: first max in (0,0),(0,1),(1,0),(1,1) order
        xp = F.pad(x.float().permute(0, 3, 1, 2), (0, 2 * Wo - W, 0, 2 * Ho - H), value=-math.inf)
        win = xp.unfold(2, 2, 2).unfold(3, 2, 2).reshape(B, C, Ho, Wo, 4)
        first = (win == win.max(-1, keepdim=True).values).float().cumsum(-1).eq(1) & (win == win.max(-1, keepdim=True).values)
        gw = first.float() * dy.float().permute(0, 3, 1, 2).unsqueeze(-1)
        gfull = gw.reshape(B, C, Ho, Wo, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, 2 * Ho, 2 * Wo)
        assert torch.equal(dx.float(), gfull[:, :, :H, :W].permute(0, 2, 3, 1))


def test_upsample_bilinear2x_add_and_backward():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(1)
    for (B, h, w, C) in [(2, 8, 8, 256), (1, 1, 1, 8), (3, 5, 7, 16)]:
        prev = bf(torch.randn(B, h, w, C, generator=g)).cuda()
        other = bf(torch.randn(B, 2 * h, 2 * w, C, generator=g)).cuda()
        out = torch.empty_like(other)
        nn.upsample_bilinear2x_add(prev, other, out)
        up = F.interpolate(prev.double().permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                           align_corners=False).permute(0, 2, 3, 1)
        ref = up + other.double()
        err = (out.double() - ref).abs() / ref.abs().clamp(min=1e-3)
        assert float(err.max()) <= 2 ** -7, float(err.max())
        dout = bf(torch.randn(B, 2 * h, 2 * w, C, generator=g)).cuda()
        dprev = torch.empty_like(prev)
        nn.upsample_bilinear2x_backward(dout, dprev)
        p = prev.double().requires_grad_(True)
        u = F.interpolate(p.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear", align_corners=False)
        (gref,) = torch.autograd.grad(u, p, dout.double().permute(0, 3, 1, 2))
        assert rel(dprev, gref) < 4e-3


def test_sep_fold_unfold():
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(2)
    ents, refs = [], []
    for (k, cin, cout) in [(1, 256, 128), (3, 128, 128), (7, 3, 128), (1, 128, 256)]:
        dw = torch.randn(k, k, cin, 1, generator=g).cuda()
        pw = torch.randn(1, 1, cin, cout, generator=g).cuda()
        weff = torch.empty(k, k, cin, cout, device="cuda")
        gweff = torch.randn(k, k, cin, cout, generator=g).cuda()
        gdw, gpw = torch.empty_like(dw), torch.empty_like(pw)
        ents.append((dw, pw, weff, gweff, gdw, gpw))
    plan = nn.SepPlan(ents, torch.device("cuda"))
    plan.fold()
    plan.unfold()
    for dw, pw, weff, gweff, gdw, gpw in ents:
        d, p = dw.double().requires_grad_(True), pw.double().requires_grad_(True)
        w = d[..., 0].unsqueeze(-1) * p[0, 0].unsqueeze(0).unsqueeze(0)
        assert rel(weff, w.detach()) < 1e-6
        a, b = torch.autograd.grad(w, (d, p), gweff.double())
        assert rel(gdw, a) < 1e-5 and rel(gpw, b) < 1e-5


@pytest.mark.parametrize("group,C", [(1, 64), (2, 64), (3, 64), (2, 2272)])
def test_bn_grouped_stats_and_backward(group, C):
    """C = 2272: more than 256 8-channel groups and not a multiple of them (the CenterNet v2
    concat, tf_hourglass_net.py:337-344) -- the uniform channel-group loop."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(3)
    B, H, W = 5, 12, 10
    x = bf(torch.randn(B, H, W, C, generator=g) * 2 + 0.5).cuda()
    gamma = (torch.rand(C, generator=g) + 0.5).cuda()
    beta = torch.randn(C, generator=g).cuda()
    stats = nn.bn_acc(B, C, "cuda")
    nn.bn_stats(x, B, H * W, C, stats)
    xd = x.double().cpu()
    sv = nn.bn_acc_value(stats).cpu()
    assert torch.allclose(sv[:, :, 0], xd.sum((1, 2)), rtol=1e-5)
    assert torch.allclose(sv[:, :, 1], (xd * xd).sum((1, 2)), rtol=1e-5)
    mr = torch.empty((B, C, 2), dtype=torch.float32, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nn.bn_finalize_grouped(stats, mr, rm, rv, B, C, H * W, group, 1e-3, 0.99)
    y = torch.empty_like(x)
    nn.bn_apply(x, mr, gamma, beta, None, y, B, H * W, C, False)
    # fp64 reference with sub-batch statistics
    xr = xd.clone().requires_grad_(True)
    outs, erm, erv = [], torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    for s in range(0, B, group):
        xs = xr[s:s + group]
        m = xs.mean((0, 1, 2))
        v = ((xs - m) ** 2).mean((0, 1, 2))
        n = xs.shape[0] * H * W
        erm = erm * 0.99 + m.detach() * 0.01
        erv = erv * 0.99 + v.detach() * n / (n - 1) * 0.01
        outs.append((xs - m) / torch.sqrt(v + 1e-3) * gamma.double().cpu() + beta.double().cpu())
    yr = torch.cat(outs)
    assert rel(y, yr.detach()) < 1e-2
    assert rel(rm, erm) < 1e-5 and rel(rv, erv) < 1e-5
    dy = bf(torch.randn(B, H, W, C, generator=g)).cuda()
    (gx,) = torch.autograd.grad(yr, xr, dy.double().cpu())
    dgamma, dbeta = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    prev = bf(torch.randn(B, H, W, C, generator=g)).cuda()
    dx = prev.clone()
    nn.bn_backward_grouped(dy, x, mr, gamma, dx, dgamma, dbeta, B, H * W, C, group, dz_beta=1.0)
    assert rel(dx, gx + prev.double().cpu()) < 1e-2
    xh = torch.cat([(xd[s:s + group] - xd[s:s + group].mean((0, 1, 2))) /
                    torch.sqrt(xd[s:s + group].var((0, 1, 2), unbiased=False) + 1e-3) for s in range(0, B, group)])
    assert rel(dgamma, (dy.double().cpu() * xh).sum((0, 1, 2))) < 1e-4
    assert rel(dbeta, dy.double().cpu().sum((0, 1, 2))) < 1e-5


def test_adam_clip_matches_oracle():
    from cvlite.train_centernet import Adam
    from cvlite.layers import ParamStore, constant
    from oracle import centernet_model_ref as cm
    st = ParamStore()
    st.add("a", (1000,), constant(0.0))
    st.add("b", (37,), constant(0.0))
    st.finalize("cuda")
    g = torch.Generator().manual_seed(4)
    st.flat.copy_(torch.randn(st.flat.numel(), generator=g).cuda())
    opt = Adam(learning_rate=1e-3).bind(st)
    P = {k: st.p(k).detach().cpu().clone() for k in ("a", "b")}
    M = {k: torch.zeros_like(v) for k, v in P.items()}
    V = {k: torch.zeros_like(v) for k, v in P.items()}
    for it in range(3):
        st.grad.zero_()                   # alignment padding of the flat buffer stays 0, as in training
        for k in P:
            st.g(k).copy_(torch.randn(P[k].numel(), generator=g).cuda() * (10.0 if it == 0 else 0.01))
        gr = {k: st.g(k).detach().cpu().clone() for k in P}
        opt.apply(st, 1.0 / 4, 1.0)
        cm.adam_step(P, gr, M, V, it, 1e-3, 4, clip=1.0)
        for k in P:
            assert torch.allclose(st.p(k).cpu(), P[k], rtol=1e-6, atol=1e-7)
    assert int(opt.iterations.item()) == 3


def test_centernet_loss_kernel():
    from cvlite import ops_targets as ot
    from oracle import centernet_model_ref as cm
    g = torch.Generator().manual_seed(5)
    B, Hs, C = 3, 16, 20
    pred = (torch.randn(B, Hs, Hs, 4 + C, generator=g) * 2).cuda()
    tg = torch.zeros(B, Hs, Hs, 4 + C)
    for b in range(B):
        for _ in range(4):
            i, j = torch.randint(0, Hs, (2,), generator=g)
            tg[b, i, j, :4] = torch.rand(4, generator=g) * 3
            tg[b, i, j, 4 + int(torch.randint(0, C, (1,), generator=g))] = 1.0
    tg = tg.cuda()
    losses, d = ot.centernet_loss(pred.view(B, -1, 4 + C), tg.view(B, -1, 4 + C), C, 2.5, 1.0)
    for b in range(B):
        p = pred[b].double().cpu().requires_grad_(True)
        c, r = cm.model_loss(tg[b].double().cpu(), p)
        assert abs(float(losses[b, 0]) - float(c)) <= 1e-5 * abs(float(c)) + 1e-4
        assert abs(float(losses[b, 1]) - float(r)) <= 1e-5 * abs(float(r)) + 1e-4
        (gp,) = torch.autograd.grad(2.5 * c + r, p)
        gd = d[b].view(Hs, Hs, -1)[..., :4 + C].double().cpu()
        assert rel(gd, gp) < 4e-3
        assert torch.all(d[b].view(Hs, Hs, -1)[..., 4 + C:] == 0)


def _small_net(C=20, seed=0, **opts):
    from cvlite.hourglass_net import HourglassNet
    return HourglassNet(C, seed=seed, **opts)


def _targets(B, Hs, C, seed):
    g = torch.Generator().manual_seed(seed)
    tg = torch.zeros(B, Hs, Hs, 4 + C)
    for b in range(B):
        for _ in range(3):
            i, j = torch.randint(0, Hs, (2,), generator=g)
            tg[b, i, j, :4] = torch.rand(4, generator=g) * 2
            tg[b, i, j, 4 + int(torch.randint(0, C, (1,), generator=g))] = 1.0
    return tg


@pytest.mark.parametrize("split", [False, True])
def test_hourglass_forward_loss_backward_vs_oracle(split, monkeypatch):
    """Whole graph, B=4 images of 128x128 in 2 BN sub-batches of 2, vs the oracle storing
    activations / weights / gradients in bf16 at the GPU path's points.  split=True lowers the
    split threshold so every 3x3 separable conv on a >= 16x16 map runs as depthwise kernel +
    pointwise GEMM (the form the bench's 256x256 / 128x128 maps take)."""
    from cvlite import hourglass_net, ops_targets as ot
    from oracle import centernet_model_ref as cm
    monkeypatch.setattr(hourglass_net, "SPLIT_MIN_HW", 256 if split else 10 ** 9)
    C, B, D, G = 20, 4, 128, 2
    net = _small_net(C, seed=1)
    params = net.store.state_dict()
    gx = torch.Generator().manual_seed(7)
    x = torch.rand(B, D, D, 3, generator=gx) * 2 - 1
    Hs = D // 4
    tg = _targets(B, Hs, C, 8)
    out = net.forward(x.cuda(), group=G)
    d_out = torch.zeros((B, Hs, Hs, net.cout_ld), dtype=torch.bfloat16, device="cuda")
    losses, _ = ot.centernet_loss(out.view(B, -1, 4 + C), tg.cuda().view(B, -1, 4 + C), C, 2.5, 1.0,
                                  d_pred=d_out.view(B, Hs * Hs, -1))
    net.backward(d_out)
    torch.cuda.synchronize()
    n_split = sum(1 for sc in net.seps() if sc.split)
    assert (n_split > 0) == split, n_split
    with cm.emulate_bf16():
        c16, r16, g16, o16 = cm.loss_and_grads(params, x, tg, C, G)
    c32, r32, g32, o32 = cm.loss_and_grads(params, x, tg, C, G)
    e_out = rel(out.cpu(), o16)
    print("out vs bf16-oracle %.4f | bf16-oracle vs fp32 %.4f" % (e_out, rel(o16, o32)))
    assert e_out < 3e-2
    lc, lr = float(losses[:, 0].sum()), float(losses[:, 1].sum())
    assert abs(lc - c16) / abs(c16) < 3e-2 and abs(lr - r16) / abs(r16) < 3e-2
    # bf16 storage alone moves the oracle's gradients by ~18% rel-L2 at this init (ReLU-mask flips
    # and sums with heavy cancellation, e.g. BN betas): bound the GPU by the oracle's own divergence
    def overall(ga, gb):
        n = d = 0.0
        for k in gb:
            n += float((ga[k].double() - gb[k].double()).norm() ** 2)
            d += float(gb[k].double().norm() ** 2)
        return math.sqrt(n / d)
    gpu = {k: net.store.g(k).detach().cpu() for k in g32}
    e16, e32, own = overall(gpu, g16), overall(gpu, g32), overall(g16, g32)
    print("grad rel-L2: gpu vs bf16-oracle %.4f, gpu vs fp32 %.4f, bf16-oracle vs fp32 %.4f" % (e16, e32, own))
    assert e32 < 1.5 * own + 0.02 and e16 < 1.5 * own + 0.02
    tot = math.sqrt(sum(float(g.double().norm() ** 2) for g in g32.values()))
    bad = []
    for k, gref in g32.items():
        if k == "cnn_block_0/bias":       # conv bias in front of a BatchNorm: gradient is exactly 0
            continue
        if float(gref.norm()) < 1e-3 * tot:
            continue
        eg, eo = rel(gpu[k], gref), rel(g16[k], gref)
        if eg > 2.0 * eo + 0.1:
            bad.append((k, round(eg, 3), round(eo, 3)))
    assert not bad, bad


@pytest.mark.parametrize("split", [False, True])
def test_hourglass_train_steps_vs_oracle(split, monkeypatch):
    """Two full device train steps (targets from boxes on the GPU, BN sub-batches of 2, Adam,
    re-pack) vs the oracle's train_step on the same targets: loss within bf16 tolerance and the
    parameter updates (Adam: ~lr per element) in rel-L2; split=True as above (the mode switch on
    the first forward re-plans the fold / pack tables before the graphs are captured)."""
    from cvlite import hourglass_net, ops_targets as ot
    from cvlite.train_centernet import CenterNetTrainer, synthetic_batch
    from oracle import centernet_model_ref as cm
    monkeypatch.setattr(hourglass_net, "SPLIT_MIN_HW", 256 if split else 10 ** 9)
    C, B, D, G = 20, 4, 128, 2
    net = _small_net(C, seed=2)
    p0 = net.store.state_dict()
    tr = CenterNetTrainer(net, B, (D, D), sub_batch_sz=G, n_max=8, use_graph=True)
    imgs, boxes, nbox = synthetic_batch(B, D, D, C, n_max=8, seed=11)
    P = {k: v.clone() for k, v in p0.items()}
    M = {k: torch.zeros_like(v) for k, v in P.items()}
    V = {k: torch.zeros_like(v) for k, v in P.items()}
    for it in range(2):
        tr.load_batch(imgs, boxes, nbox)
        losses = tr.step().double().sum(0).cpu()
        tg = tr.targets.detach().cpu()
        ref_t = ot.centernet_assign(boxes, nbox, tr.img_dim, (D, D), C, stride=4).cpu()
        assert torch.equal(tg, ref_t)
        with cm.emulate_bf16():
            c, r = cm.train_step_reference(P, M, V, it, imgs.cpu(), tg, C, G)
        assert abs(float(losses[0]) / B - c) / abs(c) < 3e-2
        if it == 0:
            m1 = _moment_rel(tr, net, M)
    # after step 1 the first moment is 0.1 * clipped(g / B): a gradient-level check (bound: the
    # gradient test above, ~18% rel-L2 from bf16 storage alone).  Step 2's gradient is taken at
    # parameters that already differ by 2*lr wherever step 1's direction flipped, so only its loss
    # and the update direction are compared.
    agree = tot = 0
    for k in P:
        dg = net.store.p(k).detach().cpu().double() - p0[k].double()
        dr = P[k].double() - p0[k].double()
        agree += int(((dg > 0) == (dr > 0)).sum())
        tot += dg.numel()
    print("Adam first-moment (step 1) rel-L2 %.4f, update sign agreement %.4f" % (m1, agree / tot))
    assert m1 < 0.3
    assert agree / tot > 0.8


def _moment_rel(tr, net, M):
    num = den = 0.0
    for k in M:
        off, n, shape = net.store.offsets[k]
        mg = tr.opt.m[off:off + n].view(shape).detach().cpu().double()
        num += float((mg - M[k].double()).norm() ** 2)
        den += float(M[k].double().norm() ** 2)
    return math.sqrt(num / den)


BUILD_OPTIONS = [dict(n_stacks=2), dict(seperable=False), dict(batch_norm=False), dict(norm_order="norm_last"),
                 dict(n_stacks=2, seperable=False, batch_norm=True, norm_order="norm_last")]


@pytest.mark.parametrize("opts", BUILD_OPTIONS, ids=lambda o: "-".join("%s=%s" % kv for kv in sorted(o.items())))
def test_hourglass_build_options_vs_oracle(opts):
    """tf_centernet_hourglass.build_model's non-default options (VERDICT r03 missing #3): stacked
    hourglasses, Conv2D (seperable=False), no BatchNormalization, norm_last -- forward output,
    losses and parameter gradients vs the oracle with bf16 storage emulated at the GPU path's
    points (same bounds as the default build's test above)."""
    from cvlite import ops_targets as ot
    from cvlite.centernet_hourglass import build_model
    from oracle import centernet_model_ref as cm
    C, B, D, G = 20, 4, 128, 2
    net = build_model(C, n_filters=64, **opts)
    params = net.store.state_dict()
    gx = torch.Generator().manual_seed(17)
    x = torch.rand(B, D, D, 3, generator=gx) * 2 - 1
    Hs = D // 4
    tg = _targets(B, Hs, C, 18)
    out = net.forward(x.cuda(), group=G)
    d_out = torch.zeros((B, Hs, Hs, net.cout_ld), dtype=torch.bfloat16, device="cuda")
    losses, _ = ot.centernet_loss(out.view(B, -1, 4 + C), tg.cuda().view(B, -1, 4 + C), C, 2.5, 1.0,
                                  d_pred=d_out.view(B, Hs * Hs, -1))
    net.backward(d_out)
    torch.cuda.synchronize()
    build = dict(n_stacks=opts.get("n_stacks", 1), seperable=opts.get("seperable", True),
                 batch_norm=opts.get("batch_norm", True), norm_order=opts.get("norm_order", "norm_first"))
    with cm.emulate_bf16():
        c16, r16, g16, o16 = cm.loss_and_grads(params, x, tg, C, G, **build)
    c32, r32, g32, o32 = cm.loss_and_grads(params, x, tg, C, G, **build)
    e_out = rel(out.cpu(), o16)
    print("%r: out vs bf16-oracle %.4f | bf16-oracle vs fp32 %.4f" % (opts, e_out, rel(o16, o32)))
    assert e_out < 3e-2
    lc, lr = float(losses[:, 0].sum()), float(losses[:, 1].sum())
    assert abs(lc - c16) / abs(c16) < 3e-2 and abs(lr - r16) / abs(r16) < 3e-2

    def overall(ga, gb):
        n = d = 0.0
        for k in gb:
            n += float((ga[k].double() - gb[k].double()).norm() ** 2)
            d += float(gb[k].double().norm() ** 2)
        return math.sqrt(n / d)
    gpu = {k: net.store.g(k).detach().cpu() for k in g32}
    assert set(gpu) == set(params)
    e16, e32, own = overall(gpu, g16), overall(gpu, g32), overall(g16, g32)
    print("grad rel-L2: gpu vs bf16-oracle %.4f, gpu vs fp32 %.4f, bf16-oracle vs fp32 %.4f" % (e16, e32, own))
    assert e32 < 1.5 * own + 0.02 and e16 < 1.5 * own + 0.02
