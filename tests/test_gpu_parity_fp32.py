"""fp32 parity mode (CVL_PRECISION=fp32, SURVEY.md §8b "Parity modes"): the detector graphs with
fp32 activations / gradients / packed weights and fp32 FMA on the GPU vs the oracle
(oracle/model_ref.py: FCOS/fcos.py:6-110 + Keras ResNet50 v1, RetinaNet/retinanet_module.py:8-159)
run in float64 on identical weights, images and targets -- no bf16 self-divergence bound.

What limits any fp32 implementation here (measured, tools/ diagnosis in DESIGN.md §parity):
the forward of a 50-layer random-init graph moves each activation by ~1e-5 relative, so a
handful of ReLU inputs within that distance of 0 land on the other side of the mask (e.g. 1 of
the 2,048 P7 tower outputs).  A flipped mask element changes the backward by O(its gradient):
the oracle itself, run in fp32 on the CPU, lands 1-4 % (rel-L2) from its float64 run on BN
gamma / beta gradients (near-cancelling sums) and 0.5 % on whole FPN-level gradients -- while
GIVEN the same masks the GPU backward matches float64 to ~1e-6 (test_fcos_fp32_tower_backward_exact).
So:
  * logits: rel-L2 and max error <= LOGIT_RTOL (damped init, the well-conditioned graph) or
    <= max(LOGIT_RTOL, NOISE_X x the fp32 oracle's own error) (the reference's Keras init);
  * per-image losses: <= max(LOSS_RTOL, the fp32 oracle's logit rel-L2) -- a loss cannot be more
    accurate than the logits it is a function of;
  * parameter gradients: the GPU's per-tensor rel-L2 errors vs float64 are no worse than the fp32
    oracle's at the median, the 90th percentile and the maximum (each within NOISE_X, or under
    GRAD_RTOL), and the flat rel-L2 over all gradients likewise;
  * test_fcos_fp32_tower_backward_exact: heads + towers backward with the GPU's own ReLU masks,
    every FPN level, within 1e-5 of float64 (no mask noise left to hide behind).
The fp32-CPU <-> fp64 distance is printed next to GPU <-> fp64 for every check."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu

LOGIT_RTOL = 1e-4        # logits: rel-L2 over each output tensor, and max |err| <= 1e-4 * max |logit|
LOSS_RTOL = 1e-5         # per-image losses (each of cls / reg / cen), relative
GRAD_RTOL = 1e-3         # parameter gradient rel-L2 (quantiles, see above)
NOISE_X = 1.5            # allowed multiple of the fp32 oracle's own error
EXACT_RTOL = 1e-5        # backward given identical ReLU masks


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def _damp_residual_gammas(net, factor=0.25):
    for k in net.store.offsets:
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(factor)


def _check_outputs(name, got, ref32, ref64, noise_rel):
    e, e_cpu = rel(got, ref64), rel(ref32, ref64)
    mx = float((got.double() - ref64.double()).abs().max()) / max(float(ref64.abs().max()), 1e-30)
    mx_cpu = float((ref32.double() - ref64.double()).abs().max()) / max(float(ref64.abs().max()), 1e-30)
    print("%s: gpu-vs-fp64 rel-L2 %.2e max %.2e | cpu-fp32-vs-fp64 %.2e max %.2e | gpu-vs-cpu-fp32 %.2e" % (
        name, e, mx, e_cpu, mx_cpu, rel(got, ref32)))
    tol, tol_mx = (max(LOGIT_RTOL, NOISE_X * e_cpu), max(LOGIT_RTOL, NOISE_X * mx_cpu)) if noise_rel else (
        LOGIT_RTOL, LOGIT_RTOL)
    ok = e <= tol and mx <= tol_mx
    return [] if ok else [("logits " + name, e, mx, tol, tol_mx)]


def _check_losses(got, l32, l64, logit_noise):
    err = ((got - l64).abs() / l64.abs().clamp(min=1e-12))
    err_cpu = ((l32.double() - l64).abs() / l64.abs().clamp(min=1e-12))
    tol = max(LOSS_RTOL, logit_noise)
    print("losses: gpu-vs-fp64 max rel %.2e (cpu fp32 %.2e), tolerance %.2e" % (
        float(err.max()), float(err_cpu.max()), tol))
    return [] if float(err.max()) <= tol else [("losses", float(err.max()), tol)]


def _perturbed(x, seed):
    """x with every element moved by +-1 ulp (fp32): another realisation of fp32 forward noise."""
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, 2, x.shape, generator=g).double() * 2 - 1
    return (x.double() * (1 + u * 2.0 ** -23)).float()


def _check_grads(grads_gpu, g64, g32s, skip_bias_before_bn=True):
    """g32s: the fp32 oracle's gradients for several realisations of fp32 noise (the images and
    their +-1-ulp perturbations): which tensors a ReLU-mask flip hits varies from one realisation
    to the next (measured: p90 1.3e-3 .. 2.8e-3 over five realisations of one RetinaNet graph),
    so the yardstick is the largest of the realisations at each quantile."""
    big = max(float(v.norm()) for v in g64.values())
    keys = [k for k, gr in g64.items()
            if not (skip_bias_before_bn and k.endswith("_conv/bias")) and float(gr.norm()) >= 1e-6 * big]
    # (conv bias in front of a training-mode BN: the true gradient is exactly 0)

    def errs(gg):
        e = np.array([rel(gg[k], g64[k]) for k in keys])
        n_err = sum(float((gg[k].double() - g64[k]).norm()) ** 2 for k in keys)
        n_ref = sum(float(g64[k].norm()) ** 2 for k in keys)
        return e, math.sqrt(n_err / n_ref)
    eg, fg = errs(grads_gpu)
    cpu = [errs(g) for g in g32s]
    fails = []
    for q in (50, 90, 100):
        a = float(np.percentile(eg, q))
        bs = [float(np.percentile(e, q)) for e, _ in cpu]
        print("gradient rel-L2 p%d: gpu %.2e | cpu-fp32 realisations %s" % (q, a, " ".join("%.2e" % b for b in bs)))
        if a > max(GRAD_RTOL, NOISE_X * max(bs)):
            fails.append(("grad p%d" % q, a, max(bs)))
    fcs = [f for _, f in cpu]
    print("flat gradient rel-L2: gpu %.2e | cpu-fp32 realisations %s" % (fg, " ".join("%.2e" % f for f in fcs)))
    if fg > max(GRAD_RTOL, NOISE_X * max(fcs)):
        fails.append(("grad flat", fg, max(fcs)))
    order = np.argsort(-eg)[:5]
    print("largest gpu errors (gpu, cpu-fp32 base, tensor):",
          [("%.2e" % eg[i], "%.2e" % cpu[0][0][i], keys[i]) for i in order])
    return fails


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


@pytest.mark.parametrize("init", ["damped", "keras"])
def test_fcos_fp32_graph_matches_reference(init):
    """FCOS ResNet-50-FPN at 256x256, bs 2: logits (reg + centerness, classes), the per-image
    (cls, reg, cen) losses and every parameter gradient vs the float64 oracle (module docstring)."""
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, seed=1, precision="fp32")
    assert net.store.act == torch.float32 and net.cls_tower[0].wf.dtype == torch.float32
    if init == "damped":
        _damp_residual_gammas(net)
    noise_rel = init == "keras"
    params = net.store.state_dict()
    x, boxes, nbox = _synth(B, D, C, 3)
    tg, reg, cls, losses = _fcos_gpu(net, x, boxes, nbox, C, B, D)
    xt = torch.from_numpy(x)
    l32, g32, reg32, cls32 = model_ref.fcos_loss_and_grads(params, xt, tg, C)
    l64, g64, reg64, cls64 = model_ref.fcos_loss_and_grads(params, xt, tg, C, dtype=torch.float64)
    g32s = [g32] + [model_ref.fcos_loss_and_grads(params, _perturbed(xt, s), tg, C)[1] for s in (1, 2)]
    fails = _check_outputs("reg", reg, reg32, reg64, noise_rel) + _check_outputs("cls", cls, cls32, cls64, noise_rel)
    fails += _check_grads({k: net.store.g(k).detach().cpu() for k in g64}, g64, g32s)
    fails += _check_losses(losses, l32, l64, max(rel(reg32, reg64), rel(cls32, cls64)))
    assert not fails, fails


def test_fcos_fp32_tower_backward_exact():
    """Keras init: the heads' and towers' data gradients of every FPN level (FCOS/fcos.py:74-110:
    per-level output convs, 4 shared 3x3 tower convs with one ReLU) on the GPU vs float64 applied
    to the GPU's own loss gradients and ReLU masks -- the parity-mode kernels, segments, pairing
    and accumulation order with the mask noise removed: EXACT_RTOL."""
    from cvlite import ops_targets as ot
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, seed=1, precision="fp32")
    x, boxes, nbox = _synth(B, D, C, 3)
    cap = {}
    orig = net.trunk_backward

    def spy(dA_top, hook=None):
        cap["dA"] = [t.detach().clone() for t in dA_top]
        cap["tw"] = [tw[-1].detach().clone() for tw in net._saved["towers"]]
        return orig(dA_top, hook=hook)
    net.trunk_backward = spy
    from cvlite import ops_nn as nn
    orig_wg = nn.conv_wgrad

    def wg_spy(d, x_, dy, dw, *a, **k):
        if dw is not None and dw.data_ptr() == net.c7_3x3.dw.data_ptr():
            cap["dF"] = dy.detach().clone()          # the towers' input gradient, all levels
        return orig_wg(d, x_, dy, dw, *a, **k)
    nn.conv_wgrad = wg_spy
    try:
        dims = torch.full((B, 2), float(D), device="cuda")
        tg, _ = ot.fcos_assign(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), dims, (D, D), C)
        reg, cls = net.forward(torch.from_numpy(x).cuda())
        P = reg.shape[1]
        d_reg = torch.zeros((B, P, 32), dtype=torch.float32, device="cuda")
        d_cls = torch.zeros((B, P, 32), dtype=torch.float32, device="cuda")
        ot.fcos_loss(reg, cls, tg, C, grad_scale=1.0, d_reg=d_reg, d_cls=d_cls)
        net.backward(d_reg, d_cls)
        torch.cuda.synchronize()
    finally:
        nn.conv_wgrad = orig_wg
    sp = {k: v.double().cpu() for k, v in net.store.state_dict().items()}

    def convT(g, name):                 # 3x3 / stride 1 / same: d input from d output
        return F.conv_transpose2d(g, sp[name + "/kernel"].permute(3, 2, 0, 1), padding=1)
    shapes, off, _ = net.layout(B, D, D)
    for l, (h, w) in enumerate(shapes):
        pts = slice(off[l], off[l] + h * w)
        rows = slice(B * off[l], B * (off[l] + h * w))
        nchw = lambda t: t[rows].cpu().double().view(B, h, w, -1).permute(0, 3, 1, 2)  # noqa: E731
        gc = d_cls.cpu()[:, pts, :C].double().reshape(B, h, w, C).permute(0, 3, 1, 2)
        gr = d_reg.cpu()[:, pts, :5].double().reshape(B, h, w, 5).permute(0, 3, 1, 2)
        dA = [nchw(cap["dA"][0]), nchw(cap["dA"][1])]
        e_head = (rel(dA[0], convT(gc, "logits_output_%d" % (l + 1))),
                  rel(dA[1], convT(gr, "reg_output_%d" % (l + 1))))
        tot = 0
        for t, pre in enumerate(("cls_layer_%d", "reg_layer_%d")):
            g = dA[t] * (nchw(cap["tw"][t]) > 0).double()
            for i in range(4, 0, -1):
                g = convT(g, pre % i)
            tot = tot + g
        e_tower = rel(nchw(cap["dF"]), tot) if l != 3 else 0.0   # P6's rows also get relu(P6)'s term
        print("level %d: head dgrad %.2e %.2e, towers %.2e" % (l, e_head[0], e_head[1], e_tower))
        assert max(e_head) <= EXACT_RTOL and e_tower <= EXACT_RTOL, (l, e_head, e_tower)


@pytest.mark.parametrize("init", ["damped", "keras"])
def test_retinanet_fp32_graph_matches_reference(init):
    """RetinaNet ResNet-50-FPN (per-(level, anchor) heads fused per level) at 256x256, bs 2, C = 8:
    same checks as FCOS (retinanet_module.py:8-159, 403-426)."""
    from cvlite import ops_targets as ot
    from cvlite.retina_net import RetinaNetNet
    from cvlite.retinanet import RetinaNet
    C, A, B, D = 8, 9, 2, 256
    net = RetinaNetNet(C, seed=4, precision="fp32")
    if init == "damped":
        _damp_residual_gammas(net)
    noise_rel = init == "keras"
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
    xt = torch.from_numpy(x)
    l32, g32, reg32, cls32 = model_ref.retina_loss_and_grads(params, xt, tgc, C, cells, A)
    l64, g64, reg64, cls64 = model_ref.retina_loss_and_grads(params, xt, tgc, C, cells, A, dtype=torch.float64)
    g32s = [g32] + [model_ref.retina_loss_and_grads(params, _perturbed(xt, s), tgc, C, cells, A)[1] for s in (1, 2)]
    fails = _check_outputs("reg", reg[..., :4 * A].cpu(), reg32, reg64, noise_rel)
    fails += _check_outputs("cls", cls[..., :A * C].cpu(), cls32, cls64, noise_rel)
    fails += _check_grads({k: net.store.g(k).detach().cpu() for k in g64}, g64, g32s)
    fails += _check_losses(losses.cpu().double(), l32, l64, max(rel(reg32, reg64), rel(cls32, cls64)))
    assert not fails, fails


def test_fcos_fp32_train_steps_match_reference_step():
    """Two FCOSTrainer steps in the parity mode (graph replay: targets, forward, loss, backward,
    /bs, clip_by_global_norm, Keras SGD; FCOS/train_fcos.py:107-185) vs train_step_reference in
    float64 on the same targets, damped init (the keras-init graph is covered, against fp32 noise,
    by the graph tests above): the momentum buffers (= the clipped, scaled gradient history) within
    GRAD_RTOL (rel-L2 over all parameters) of float64, and the weights exactly the Keras fp32
    update of the GPU's own momentum, w = fl32(w_prev + v) (the weight-update rel-L2 vs float64 is
    printed: on top of the momentum error it carries fp32 weight-storage rounding, updates of
    ~1e-7 relative on O(0.05) weights)."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, D, lr = 20, 2, 256, 5e-4
    net = FCOSNet(C, seed=2, precision="fp32")
    _damp_residual_gammas(net)
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
    st = net.store
    for it in range(2):
        p_prev = {k: st.p(k).detach().cpu().clone() for k in names}
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
        # weights are stored in fp32 (as the reference's): compare updates as stored, i.e. the
        # float64 step rounded to the fp32 weight, minus the fp32 start
        dw = {k: st.p(k).detach().cpu().double() - p0[k].double() for k in names}
        d64 = {k: P64[k].float().double() - p0[k].double() for k in names}
        e_m, e_w = flat_rel(mom, M64), flat_rel(dw, d64)
        print("step %d (grad norm %.4f): momentum rel-L2 %.2e, weight update rel-L2 %.2e" % (it + 1, norm, e_m, e_w))
        assert e_m <= GRAD_RTOL
        for k in names:
            torch.testing.assert_close(st.p(k).detach().cpu(), p_prev[k] + mom[k], rtol=0, atol=0)
