"""fp32 parity mode (CVL_PRECISION=fp32, SURVEY.md §8b "Parity modes"): the detector graphs with
fp32 activations / gradients / packed weights and fp32 FMA on the GPU vs the fp32 oracle
(oracle/model_ref.py: FCOS/fcos.py:6-110 + Keras ResNet50 v1, RetinaNet/retinanet_module.py:8-159)
on identical weights, images and targets, at the REFERENCE'S OWN init (Keras glorot, undamped) --
no bf16 self-divergence bound: the tolerances are fixed numbers, written in each test.

The oracle is also run in float64; the distance fp32-CPU <-> fp64 is printed next to GPU <-> fp64
so a reader can see how much of the GPU's deviation is plain fp32 summation-order noise (amplified
by the random-init graph) and how much would be the kernels'."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu

LOGIT_RTOL = 1e-4        # logits: rel-L2 over each output tensor, and max |err| <= 1e-4 * max |logit|
LOSS_RTOL = 1e-5         # per-image losses (each of cls / reg / cen), relative
GRAD_RTOL = 1e-3         # every parameter gradient tensor, rel-L2


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def _check_outputs(name, got, ref32, ref64):
    e, e_cpu = rel(got, ref64), rel(ref32, ref64)
    mx = float((got.double() - ref64.double()).abs().max()) / max(float(ref64.abs().max()), 1e-30)
    print("%s: gpu-vs-fp64 rel-L2 %.2e max %.2e | cpu-fp32-vs-fp64 %.2e | gpu-vs-cpu-fp32 %.2e" % (
        name, e, mx, e_cpu, rel(got, ref32)))
    assert e <= LOGIT_RTOL and mx <= LOGIT_RTOL, (name, e, mx)


def _check_grads(grads_gpu, g64, skip_bias_before_bn=True):
    big = max(float(v.norm()) for v in g64.values())
    worst = []
    for k, gr in g64.items():
        if skip_bias_before_bn and k.endswith("_conv/bias"):
            continue              # conv bias in front of a training-mode BN: the true gradient is exactly 0
        if float(gr.norm()) < 1e-6 * big:
            continue
        worst.append((rel(grads_gpu[k], gr), k))
    worst.sort(reverse=True)
    print("worst gradient tensors (rel-L2 vs fp64 oracle):", [(round(e, 6), k) for e, k in worst[:4]])
    assert worst[0][0] <= GRAD_RTOL, worst[:4]


def _synth(B, D, C, seed, nmax=6):
    rng = np.random.default_rng(seed)
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = np.zeros(B, np.int32)
    for b in range(B):
        n = int(rng.integers(1, nmax + 1))
        nbox[b] = n
        for i in range(n):
            h, w = np.exp(rng.uniform(np.log(12 / D), np.log(0.9), 2))
            boxes[b, i] = [rng.uniform(h / 2, 1 - h / 2), rng.uniform(w / 2, 1 - w / 2), h, w, rng.integers(0, C)]
    x = rng.uniform(-1, 1, size=(B, D, D, 3)).astype(np.float32)
    return x, boxes, nbox


CONV_CASES = [  # (B, H, W, Cin, Cout, k, stride, pad, relu_in)
    (2, 16, 16, 64, 64, 3, 1, "same", False),
    (2, 16, 16, 128, 256, 1, 2, "same", False),
    (1, 9, 7, 32, 48, 3, 2, "same", True),
    (2, 19, 21, 3, 64, 7, 2, 3, False),
    (3, 8, 8, 256, 20, 3, 1, "same", False),
]


def _pads(n, k, s, mode):
    if mode == "same":
        out = -(-n // s)
        t = max((out - 1) * s + k - n, 0)
        return out, t // 2, t - t // 2
    p = int(mode)
    return (n + 2 * p - k) // s + 1, p, p


@pytest.mark.parametrize("case", CONV_CASES)
def test_fp32_conv_fwd_dgrad_wgrad_vs_fp64(case):
    """The parity-mode conv (cvl_conv_desc.prec = CVL_PREC_F32: fwd, data gradient incl. stride 2
    and the 7x7/2 stem, weight gradient) vs float64 torch on the same fp32 operands: 2e-6."""
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout, k, s, pad, relu_in = case
    g = torch.Generator().manual_seed(H * W + Cin)
    x = torch.randn(B, H, W, Cin, generator=g)
    w = torch.randn(k, k, Cin, Cout, generator=g) * (k * k * Cin) ** -0.5
    b = torch.randn(Cout, generator=g)
    Ho, pt, pb = _pads(H, k, s, pad)
    Wo, pl, pr = _pads(W, k, s, pad)
    npad = (Cout + 31) // 32 * 32
    cin_pad = (Cin + 31) // 32 * 32
    wf = torch.empty((npad, k * k * Cin), dtype=torch.float32, device="cuda")
    wd = torch.empty((cin_pad, k * k * npad), dtype=torch.float32, device="cuda")
    plan = nn.PackPlan([(w.cuda().contiguous(), k * k, Cin, Cout, Cin, npad, wf, cin_pad, npad, wd)], "cuda")
    plan.run()
    xd = x.double().permute(0, 3, 1, 2)
    xin = F.relu(xd) if relu_in else xd
    wt = w.double().permute(3, 2, 0, 1).requires_grad_(True)
    xr = xin.clone().requires_grad_(True)
    y = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wt, b.double(), s)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64).float().double()
    (y * dy).sum().backward()
    out = torch.zeros((B, Ho, Wo, Cout), device="cuda")
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, Cout, [nn.seg(Ho, Wo, H, W, wf, b.cuda())],
                     relu_in=relu_in)
    nn.conv_igemm(d, x.cuda(), out)
    assert d.prec == nn.PREC_F32
    assert rel(out.cpu().permute(0, 3, 1, 2), y.detach()) <= 2e-6
    dyg = dy.float().permute(0, 2, 3, 1).contiguous().cuda()
    dw = torch.zeros((k, k, Cin, Cout), device="cuda")
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, Cout, [nn.seg(Ho, Wo, H, W, wf, None)],
                     relu_in=relu_in)
    nn.conv_wgrad(d, x.cuda(), dyg, dw)
    assert rel(dw.cpu().permute(3, 2, 0, 1), wt.grad) <= 2e-6
    if not relu_in:
        dx = torch.zeros((B, H, W, Cin), device="cuda")
        dd = nn.make_desc(nn.DGRAD, B, npad, k, k, s, pt, pl, cin_pad, Cin, Cin, [nn.seg(H, W, Ho, Wo, wd, None)])
        dyp = torch.zeros((B, Ho, Wo, npad), device="cuda")
        dyp[..., :Cout] = dyg
        nn.conv_igemm(dd, dyp, dx)
        assert rel(dx.cpu().permute(0, 3, 1, 2), xr.grad) <= 2e-6


def _fcos_gpu(net, x, boxes, nbox, C, B, D):
    from cvlite import ops_targets as ot
    dims = torch.full((B, 2), float(D), device="cuda")
    tg, _ = ot.fcos_assign(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), dims, (D, D), C)
    for b in range(B):
        outs, _ = fcos_ref.format_data(boxes[b, :nbox[b]], np.array([D, D], np.float32), C, img_pad=(D, D))
        np.testing.assert_array_equal(tg[b].cpu().numpy(), fcos_ref.pack_targets(outs))
    reg, cls = net.forward(torch.from_numpy(x).cuda())
    P = reg.shape[1]
    d_reg = torch.zeros((B, P, 32), dtype=torch.float32, device="cuda")
    d_cls = torch.zeros((B, P, 32), dtype=torch.float32, device="cuda")
    losses, _, _ = ot.fcos_loss(reg, cls, tg, C, grad_scale=1.0, d_reg=d_reg, d_cls=d_cls)
    net.backward(d_reg, d_cls)
    torch.cuda.synchronize()
    return tg.cpu(), reg[..., :5].cpu(), cls[..., :C].cpu(), losses.cpu().double()


def test_fcos_fp32_graph_matches_reference_at_keras_init():
    """FCOS ResNet-50-FPN at 256x256, bs 2, the reference's Keras glorot init (not damped): logits
    (reg + centerness, classes) within LOGIT_RTOL, the per-image (cls, reg, cen) losses within
    LOSS_RTOL and every parameter gradient within GRAD_RTOL of the oracle (float64 run)."""
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, seed=1, precision="fp32")
    assert net.store.act == torch.float32 and net.cls_tower[0].wf.dtype == torch.float32
    params = net.store.state_dict()
    x, boxes, nbox = _synth(B, D, C, 3)
    tg, reg, cls, losses = _fcos_gpu(net, x, boxes, nbox, C, B, D)
    l32, g32, reg32, cls32 = model_ref.fcos_loss_and_grads(params, torch.from_numpy(x), tg, C)
    l64, g64, reg64, cls64 = model_ref.fcos_loss_and_grads(params, torch.from_numpy(x), tg, C, dtype=torch.float64)
    _check_outputs("reg", reg, reg32, reg64)
    _check_outputs("cls", cls, cls32, cls64)
    el = float(((losses - l64).abs() / l64.abs().clamp(min=1e-12)).max())
    print("losses: gpu-vs-fp64 max rel %.2e (cpu fp32 %.2e)" % (
        el, float(((l32.double() - l64).abs() / l64.abs().clamp(min=1e-12)).max())))
    assert el <= LOSS_RTOL
    _check_grads({k: net.store.g(k).detach().cpu() for k in g64}, g64)


def test_retinanet_fp32_graph_matches_reference_at_keras_init():
    """RetinaNet ResNet-50-FPN (per-(level, anchor) heads fused per level) at 256x256, bs 2, C = 8,
    Keras init: same fixed tolerances as FCOS (retinanet_module.py:8-159, 403-426)."""
    from cvlite import ops_targets as ot
    from cvlite.retina_net import RetinaNetNet
    from cvlite.retinanet import RetinaNet
    C, A, B, D = 8, 9, 2, 256
    net = RetinaNetNet(C, seed=4, precision="fp32")
    params = net.store.state_dict()
    rn = RetinaNet(C, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
    x, boxes, nbox = _synth(B, D, C, 9, nmax=8)
    dims = torch.full((B, 2), float(D), device="cuda")
    tg, _ = rn.format_data_batched(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), dims, D)
    shapes, off, P = net.layout(B, D, D)
    cells = [h * w for h, w in shapes]
    reg, cls = net.forward(torch.from_numpy(x).cuda())
    d_reg = torch.zeros((B, P, net.reg_ld), dtype=torch.float32, device="cuda")
    d_cls = torch.zeros((B, P, net.cls_ld), dtype=torch.float32, device="cuda")
    losses = ot.retina_loss(reg, cls, tg, cells, A, C, grad_scale=1.0, d_reg=d_reg, d_cls=d_cls)
    net.backward(d_reg, d_cls)
    torch.cuda.synchronize()
    tgc = tg.cpu()
    l32, g32, reg32, cls32 = model_ref.retina_loss_and_grads(params, torch.from_numpy(x), tgc, C, cells, A)
    l64, g64, reg64, cls64 = model_ref.retina_loss_and_grads(params, torch.from_numpy(x), tgc, C, cells, A,
                                                             dtype=torch.float64)
    _check_outputs("reg", reg[..., :4 * A].cpu(), reg32, reg64)
    _check_outputs("cls", cls[..., :A * C].cpu(), cls32, cls64)
    lg = losses.cpu().double()
    el = float(((lg - l64).abs() / l64.abs().clamp(min=1e-12)).max())
    print("losses: gpu-vs-fp64 max rel %.2e" % el)
    assert el <= LOSS_RTOL
    _check_grads({k: net.store.g(k).detach().cpu() for k in g64}, g64)


def test_fcos_fp32_train_steps_match_reference_step():
    """Two FCOSTrainer steps in the parity mode (graph replay: targets, forward, loss, backward,
    /bs, clip_by_global_norm, Keras SGD; FCOS/train_fcos.py:107-185) vs train_step_reference in
    float64 on the same targets, Keras init: momentum buffers and weight updates within GRAD_RTOL
    (rel-L2 over all parameters)."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, D, lr = 20, 2, 256, 5e-4
    net = FCOSNet(C, seed=2, precision="fp32")
    p0 = net.store.state_dict()
    tr = FCOSTrainer(net, B, (D, D), init_lr=lr, use_graph=True)
    assert tr.d_reg.dtype == torch.float32
    imgs, boxes, nbox = synthetic_batch(B, D, D, C, seed=31)
    P64 = {k: v.double().clone() for k, v in p0.items()}
    M64 = {k: torch.zeros_like(v) for k, v in P64.items()}
    names = list(p0)

    def flat_rel(a, b):
        n = sum(float((a[k].double() - b[k]).norm() ** 2) for k in names)
        return math.sqrt(n / sum(float(b[k].norm() ** 2) for k in names))
    for it in range(2):
        tr.load_batch(imgs, boxes, nbox)
        tr.step()
        torch.cuda.synchronize()
        tg = tr.targets.detach().cpu()
        # the reference step in float64 (params / momentum kept float64)
        bs = B
        acc = {k: torch.zeros_like(v) for k, v in P64.items()}
        for b in range(bs):
            _, g, _, _ = model_ref.fcos_loss_and_grads(P64, imgs[b:b + 1].cpu(), tg[b:b + 1], C, dtype=torch.float64)
            for k, v in g.items():
                acc[k] += v
        norm = math.sqrt(sum(float(((v / bs) ** 2).sum()) for v in acc.values()))
        sc = 1.0 / max(norm, 1.0)
        for k in names:
            M64[k].mul_(0.9).sub_(float(np.float32(lr)) * acc[k] / bs * sc)
            P64[k].add_(M64[k])
        st = net.store
        mom = {k: st.mom[st.offsets[k][0]:st.offsets[k][0] + st.offsets[k][1]].view(st.offsets[k][2]).cpu()
               for k in names}
        dw = {k: st.p(k).detach().cpu().double() - p0[k].double() for k in names}
        d64 = {k: P64[k] - p0[k].double() for k in names}
        e_m, e_w = flat_rel(mom, M64), flat_rel(dw, d64)
        print("step %d (grad norm %.4f): momentum rel-L2 %.2e, weight update rel-L2 %.2e" % (it + 1, norm, e_m, e_w))
        assert e_m <= GRAD_RTOL and e_w <= GRAD_RTOL
