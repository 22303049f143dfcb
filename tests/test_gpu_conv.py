"""GPU parity of the segmented implicit-GEMM conv (fwd / dgrad / wgrad) against a torch fp64
reference of the same TF-padded convolution on the same bf16-rounded operands.
Tolerances: bf16 outputs rtol/atol 1e-2 (one bf16 rounding of the result); fp32 outputs 1e-4."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _pads(n, k, s, mode):
    if mode == "same":
        out = -(-n // s)
        t = max((out - 1) * s + k - n, 0)
        return out, t // 2, t - t // 2
    p = int(mode)
    return (n + 2 * p - k) // s + 1, p, p


def ref_conv(x, w, b, stride, pad):
    """x NHWC, w HWIO (fp64) -> NHWC fp64, TF 'same' or explicit pad."""
    k = w.shape[0]
    Ho, pt, pb = _pads(x.shape[1], k, stride, pad)
    Wo, pl, pr = _pads(x.shape[2], k, stride, pad)
    xn = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    y = F.conv2d(xn, w.permute(3, 2, 0, 1), b, stride)
    return y.permute(0, 2, 3, 1)


@pytest.fixture(params=["base", "l", "l256", "x32"])
def kern(request, dispatch):
    """Run a test through the 128-row register-staged kernel ("base"), the 256-row LDS-DMA kernel
    ("l", normally taken only by launches with >= 128 tiles; 128/64-wide N tiles), its
    256x256-tile form ("l256", Npad % 256 == 0 only) and the 256x256 32-deep-K ring kernel ("x32",
    the default for those launches).  Weight gradients: "base" runs the 128-wide k-tile kernel,
    "l"/"l256" the row-table LDS-DMA kernel (conv_wgrad_l.hip), "x32" the default dispatch
    (conv_wgrad_x.hip where Npad % 256 == 0)."""
    p = request.param
    dispatch("no_h", "wg_no_h")        # the halo kernels have their own tests (test_gpu_conv_h.py)
    if p in ("l", "l256", "x32"):
        dispatch("l_min_tiles=1")
    if p == "l":
        dispatch("no_256")
    if p in ("l256", "x32"):
        dispatch("l256_min_tiles=1")
    if p == "l256":
        dispatch("no_x")
    if p != "x32":
        dispatch("wg_no_x")
    if p == "base":
        dispatch("no_l", "wg_no_l")
    return request.param


def rnd(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen, dtype=torch.float64) * scale).to(BF).to(torch.float64)


def packs(w, cin_k=None, npad=None, cout_pad=None):
    from cvlite import ops_nn as nn
    k, _, cin, cout = w.shape
    cin_k = cin if cin_k is None else cin_k
    npad = npad or max(32, (cout + 31) // 32 * 32)
    cout_pad = cout_pad or npad
    cin_pad = (cin + 31) // 32 * 32
    wf = torch.empty((npad, k * k * cin_k), dtype=BF, device="cuda")
    wd = torch.empty((cin_pad, k * k * cout_pad), dtype=BF, device="cuda")
    nn.pack_conv_weights(w.float().cuda().contiguous(), k, k, cin, cout, cin_k, npad, wf, cin_pad, cout_pad, wd)
    return wf, wd, npad, cout_pad, cin_pad


CASES = [  # (B, H, W, Cin, Cout, k, stride, pad)
    (2, 16, 16, 64, 64, 3, 1, "same"),
    (2, 16, 16, 128, 256, 1, 2, "same"),
    (1, 9, 7, 32, 32, 3, 2, "same"),
    (3, 8, 8, 256, 96, 3, 1, "same"),
    (2, 12, 10, 64, 128, 1, 1, "same"),
    (1, 16, 16, 2048 // 8, 256, 3, 2, "same"),
    (2, 19, 21, 32, 64, 7, 2, 3),
]


@pytest.mark.parametrize("case", CASES)
def test_conv_fwd(case, kern):
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout, k, s, pad = case
    g = torch.Generator().manual_seed(sum(c for c in case if isinstance(c, int)))
    x = rnd(B, H, W, Cin, gen=g)
    w = rnd(k, k, Cin, Cout, scale=(k * k * Cin) ** -0.5, gen=g)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    ref = ref_conv(x, w, b, s, pad)
    Ho, Wo = ref.shape[1], ref.shape[2]
    _, pt, _ = _pads(H, k, s, pad)
    _, pl, _ = _pads(W, k, s, pad)
    wf, _, npad, _, _ = packs(w)
    bias = torch.zeros(npad, dtype=torch.float32, device="cuda")
    bias[:Cout] = b.float().cuda()
    xg = x.to(BF).cuda()
    # bf16 output + relu + BN stats
    out = torch.zeros((B, Ho, Wo, Cout), dtype=BF, device="cuda")
    stats = nn.bn_acc(B, Cout, "cuda")
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, Cout, [nn.seg(Ho, Wo, H, W, wf, bias)],
                     relu_out=True)
    hw = Ho * Wo
    stats_ok = hw % 128 == 0 or (128 % hw == 0 and hw % 4 == 0)
    nn.conv_igemm(d, xg, out, stats if stats_ok else None)
    torch.testing.assert_close(out.double().cpu(), ref.clamp(min=0), rtol=1e-2, atol=1e-2)
    if stats_ok:
        o = out.double().cpu()
        st = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
        torch.testing.assert_close(nn.bn_acc_value(stats).cpu(), st, rtol=1e-5, atol=1e-3)
    # fp32 output into a wider buffer at a channel offset, accumulate (beta = 1), relu on load
    ld = Cout + 16
    out32 = torch.randn((B, Ho, Wo, ld), dtype=torch.float32, device="cuda")
    before = out32.clone()
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, ld, [nn.seg(Ho, Wo, H, W, wf, bias)],
                     dst_coff=8, dst_f32=True, relu_in=True, beta=1.0)
    nn.conv_igemm(d, xg, out32)
    ref2 = ref_conv(x.clamp(min=0), w, b, s, pad)
    exp = before.double().cpu()
    exp[..., 8:8 + Cout] += ref2
    torch.testing.assert_close(out32.double().cpu(), exp, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("case", CASES[:6])
def test_conv_dgrad_wgrad(case, kern):
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout, k, s, pad = case
    g = torch.Generator().manual_seed(7 + sum(c for c in case if isinstance(c, int)))
    x = rnd(B, H, W, Cin, gen=g).requires_grad_(True)
    w = rnd(k, k, Cin, Cout, scale=(k * k * Cin) ** -0.5, gen=g).requires_grad_(True)
    y = ref_conv(x, w, None, s, pad)
    dy = rnd(*y.shape, gen=g)
    y.backward(dy)
    Ho, Wo = y.shape[1], y.shape[2]
    _, pt, _ = _pads(H, k, s, pad)
    _, pl, _ = _pads(W, k, s, pad)
    wf, wd, npad, cout_pad, cin_pad = packs(w.detach())
    dyg = torch.zeros((B, Ho, Wo, cout_pad), dtype=BF, device="cuda")
    dyg[..., :Cout] = dy.to(BF).cuda()
    # dgrad
    dx = torch.empty((B, H, W, Cin), dtype=BF, device="cuda")
    d = nn.make_desc(nn.DGRAD, B, cout_pad, k, k, s, pt, pl, cin_pad, Cin, Cin, [nn.seg(H, W, Ho, Wo, wd)])
    nn.conv_igemm(d, dyg, dx)
    torch.testing.assert_close(dx.double().cpu(), x.grad, rtol=1e-2, atol=2e-2)
    # accumulate (beta = 1) into an existing gradient (residual-branch form)
    old = torch.randn((B, H, W, Cin), generator=g).to(BF)
    dx2 = old.cuda()
    d = nn.make_desc(nn.DGRAD, B, cout_pad, k, k, s, pt, pl, cin_pad, Cin, Cin, [nn.seg(H, W, Ho, Wo, wd)], beta=1.0)
    nn.conv_igemm(d, dyg, dx2)
    torch.testing.assert_close(dx2.double().cpu(), x.grad + old.double(), rtol=1e-2, atol=3e-2)
    # wgrad
    dw = torch.zeros((k, k, Cin, Cout), dtype=torch.float32, device="cuda")
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, cout_pad, [nn.seg(Ho, Wo, H, W, wf)])
    nn.conv_wgrad(d, x.detach().to(BF).cuda(), dyg, dw)
    scale = w.grad.abs().max().item()
    torch.testing.assert_close(dw.double().cpu(), w.grad, rtol=1e-4, atol=1e-5 * scale)


def test_conv_segments_packed_levels(kern):
    """Five level maps in one packed level-major buffer through one shared-weight launch, and the
    per-level-weights head form writing an image-major [B, P, ld] fp32 buffer."""
    from cvlite import ops_nn as nn
    B, C = 3, 64
    shapes = [(16, 16), (8, 8), (4, 4), (2, 2), (1, 1)]
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    g = torch.Generator().manual_seed(3)
    maps = [rnd(B, h, w, C, gen=g) for h, w in shapes]
    packed = torch.cat([m.reshape(-1, C) for m in maps], 0).to(BF).cuda()
    w = rnd(3, 3, C, C, scale=(9 * C) ** -0.5, gen=g)
    wf, wd, npad, _, _ = packs(w)
    segs = [nn.seg(h, ww, h, ww, wf, None, src_base=B * off[l], dst_base=B * off[l]) for l, (h, ww) in enumerate(shapes)]
    out = torch.empty_like(packed)
    nn.conv_igemm(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, npad, C, C, segs), packed, out)
    for l, (h, ww) in enumerate(shapes):
        got = out[B * off[l]:B * off[l] + B * h * ww].reshape(B, h, ww, C).double().cpu()
        torch.testing.assert_close(got, ref_conv(maps[l], w, None, 1, "same"), rtol=1e-2, atol=1e-2)
    # wgrad over all levels == sum of per-level wgrads
    dy = rnd(B * P, C, gen=g).to(BF).cuda()
    dw = torch.zeros((3, 3, C, C), dtype=torch.float32, device="cuda")
    nn.conv_wgrad(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, npad, C, C, segs), packed, dy, dw)
    ref = torch.zeros(3, 3, C, C, dtype=torch.float64)
    for l, (h, ww) in enumerate(shapes):
        wl = w.clone().requires_grad_(True)
        y = ref_conv(maps[l], wl, None, 1, "same")
        y.backward(dy[B * off[l]:B * off[l] + B * h * ww].reshape(B, h, ww, C).double().cpu())
        ref += wl.grad
    torch.testing.assert_close(dw.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    # heads: per-level weights, fp32 into [B, P, 32] (n_store 20)
    Cn = 20
    hw_ = [rnd(3, 3, C, Cn, scale=0.05, gen=g) for _ in shapes]
    hb = [torch.randn(Cn, generator=g, dtype=torch.float64) for _ in shapes]
    pk = [packs(x) for x in hw_]
    biases = []
    for b in hb:
        t = torch.zeros(32, dtype=torch.float32, device="cuda")
        t[:Cn] = b.float().cuda()
        biases.append(t)
    segs = [nn.seg(h, ww, h, ww, pk[l][0], biases[l], src_base=B * off[l], dst_base=off[l], dst_img=P)
            for l, (h, ww) in enumerate(shapes)]
    res = torch.zeros((B, P, 32), dtype=torch.float32, device="cuda")
    nn.conv_igemm(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, 32, Cn, 32, segs, dst_f32=True), packed, res)
    for l, (h, ww) in enumerate(shapes):
        got = res[:, off[l]:off[l] + h * ww, :Cn].reshape(B, h, ww, Cn).double().cpu()
        torch.testing.assert_close(got, ref_conv(maps[l], hw_[l], hb[l], 1, "same"), rtol=1e-4, atol=1e-4)
    assert not res[..., Cn:].any()
    # head dgrad with per-level dgrad packs back into the packed level-major buffer
    dres = torch.zeros((B, P, 32), dtype=BF, device="cuda")
    dres[..., :Cn] = torch.randn((B, P, Cn), generator=g).to(BF).cuda()
    segs = [nn.seg(h, ww, h, ww, pk[l][1], None, src_base=off[l], src_img=P, dst_base=B * off[l])
            for l, (h, ww) in enumerate(shapes)]
    dpk = torch.empty_like(packed)
    nn.conv_igemm(nn.make_desc(nn.DGRAD, B, 32, 3, 3, 1, 1, 1, C, C, C, segs), dres, dpk)
    for l, (h, ww) in enumerate(shapes):
        xl = maps[l].clone().requires_grad_(True)
        y = ref_conv(xl, hw_[l], None, 1, "same")
        y.backward(dres[:, off[l]:off[l] + h * ww, :Cn].reshape(B, h, ww, Cn).double().cpu())
        got = dpk[B * off[l]:B * off[l] + B * h * ww].reshape(B, h, ww, C).double().cpu()
        torch.testing.assert_close(got, xl.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("case", [  # (B, H, W, Cin, Cout, k, stride): c6 and conv5-stage shapes
    (16, 16, 16, 2048, 256, 3, 2),
    (16, 16, 16, 512, 512, 3, 1),
    (16, 16, 16, 2048, 512, 1, 1),
])
def test_conv_splitk_matches_unsplit(case):
    """Small-M / large-K launches take the split-K path (fp32 partial slabs + finishing pass) when
    a workspace is given; without one the single-pass kernel runs.  Both must agree (and with fp64)."""
    import ctypes
    from cvlite import _lib, ops_nn as nn
    B, H, W, Cin, Cout, k, s = case
    g = torch.Generator().manual_seed(Cin + Cout + k)
    x = rnd(B, H, W, Cin, gen=g)
    w = rnd(k, k, Cin, Cout, scale=(k * k * Cin) ** -0.5, gen=g)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    ref = ref_conv(x, w, b, s, "same")
    Ho, Wo = ref.shape[1], ref.shape[2]
    _, pt, _ = _pads(H, k, s, "same")
    wf, _, npad, _, _ = packs(w)
    bias = b.float().cuda()
    xg = x.to(BF).cuda()
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pt, npad, Cout, Cout, [nn.seg(Ho, Wo, H, W, wf, bias)],
                     relu_out=True)
    assert _lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(d)) > 16, "shape should split"
    outs, stats = [], []
    for split in (True, False):
        out = torch.zeros((B, Ho, Wo, Cout), dtype=BF, device="cuda")
        st = nn.bn_acc(B, Cout, "cuda")
        if split:
            nn.conv_igemm(d, xg, out, st)
        else:
            _lib.call("cvl_conv_igemm", ctypes.byref(d), nn.ptr(xg), nn.ptr(out), nn.ptr(st), None, 0,
                      nn.stream())
        outs.append(out.double().cpu())
        stats.append(nn.bn_acc_value(st).cpu())
    torch.testing.assert_close(outs[0], ref.clamp(min=0), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(stats[0], stats[1], rtol=5e-3, atol=1e-1)  # bf16 ulp flips
    o = outs[0]
    torch.testing.assert_close(stats[0], torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1),
                               rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("case", [  # (B, H, W, Cin, Cout, k, stride): >= 1024 reduction rows
    (4, 32, 32, 64, 128, 3, 1),       # K = 576: partial 256-wide k tile, taps straddle a tile
    (4, 32, 32, 256, 256, 3, 2),
    (2, 64, 64, 256, 512, 1, 2),
    (3, 40, 24, 128, 128, 3, 1),      # rows not a multiple of the 128-row granule
    (16, 128, 128, 64, 256, 1, 1),    # ResNet conv2 1x1, K = 64: hundreds of split-M slabs
    (8, 64, 64, 256, 64, 1, 1),       # 64-channel outputs: half of each 128-wide tile idle
    (4, 64, 64, 64, 64, 1, 1),
    (2, 128, 128, 192, 64, 1, 1),     # the stem's im2col GEMM shape (K = 192 = 128 + 64)
])
def test_conv_wgrad_large(case, kern):
    """Weight gradient at sizes that take the 128x256 LDS-DMA kernel (and, with kern == "base",
    the 128x128 one) vs torch fp64; split-M slabs and beta accumulation."""
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout, k, s = case
    g = torch.Generator().manual_seed(B + H + Cin + Cout + k)
    x = rnd(B, H, W, Cin, gen=g)
    w = rnd(k, k, Cin, Cout, scale=(k * k * Cin) ** -0.5, gen=g).requires_grad_(True)
    y = ref_conv(x, w, None, s, "same")
    dy = rnd(*y.shape, gen=g)
    y.backward(dy)
    Ho, Wo = y.shape[1], y.shape[2]
    _, pt, _ = _pads(H, k, s, "same")
    _, pl, _ = _pads(W, k, s, "same")
    wf, _, npad, cout_pad, _ = packs(w.detach())
    dyg = torch.zeros((B, Ho, Wo, cout_pad), dtype=BF, device="cuda")
    dyg[..., :Cout] = dy.to(BF).cuda()
    old = torch.randn((k, k, Cin, Cout), generator=g).float().cuda()
    dw = old.clone()
    d = nn.make_desc(nn.FWD, B, Cin, k, k, s, pt, pl, npad, Cout, cout_pad, [nn.seg(Ho, Wo, H, W, wf)])
    nn.conv_wgrad(d, x.to(BF).cuda(), dyg, dw, beta=0.5)
    exp = w.grad + 0.5 * old.double().cpu()
    scale = w.grad.abs().max().item()
    torch.testing.assert_close(dw.double().cpu(), exp, rtol=1e-4, atol=1e-5 * scale)


def test_conv_wgrad_large_segments(kern):
    """Shared-weight wgrad over five packed levels (the FCOS tower form) at a size that takes the
    large kernel: equals the sum of the per-level weight gradients."""
    from cvlite import ops_nn as nn
    B, C = 4, 128
    shapes = [(16, 16), (8, 8), (4, 4), (2, 2), (1, 1)]
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    g = torch.Generator().manual_seed(5)
    maps = [rnd(B, h, w, C, gen=g) for h, w in shapes]
    packed = torch.cat([m.reshape(-1, C) for m in maps], 0).to(BF).cuda()
    w = rnd(3, 3, C, C, scale=(9 * C) ** -0.5, gen=g)
    wf, _, npad, _, _ = packs(w)
    segs = [nn.seg(h, ww, h, ww, wf, None, src_base=B * off[l], dst_base=B * off[l]) for l, (h, ww) in enumerate(shapes)]
    dy = rnd(B * P, C, gen=g).to(BF).cuda()
    dw = torch.zeros((3, 3, C, C), dtype=torch.float32, device="cuda")
    nn.conv_wgrad(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, npad, C, C, segs), packed, dy, dw)
    ref = torch.zeros(3, 3, C, C, dtype=torch.float64)
    for l, (h, ww) in enumerate(shapes):
        wl = w.clone().requires_grad_(True)
        y = ref_conv(maps[l], wl, None, 1, "same")
        y.backward(dy[B * off[l]:B * off[l] + B * h * ww].reshape(B, h, ww, C).double().cpu())
        ref += wl.grad
    torch.testing.assert_close(dw.double().cpu(), ref, rtol=1e-4, atol=1e-4)


def _tower_pair_case(B, C, shapes, seed):
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    g = torch.Generator().manual_seed(seed)
    xs = rnd(2 * B * P, C, gen=g)
    dys = rnd(2 * B * P, C, gen=g)
    return off, P, xs, dys


@pytest.mark.parametrize("shared_x", [False, True])
@pytest.mark.parametrize("variant", ["wx", "fallback"])
def test_conv_wgrad_grouped_tower_pair(shared_x, variant, dispatch):
    """cvl_conv_wgrad_grouped in the paired-tower form (fcos.py:16-27, 76-101): 10 segments = 2 towers
    x 5 levels, group g -> dW_g, dY rows of tower t at t*B*P; the source is either the paired
    activation buffer (layers 1-3) or one map both towers read (layer 0, shared_x).  "fallback"
    runs one single-group launch per group.  Reference: per level and tower, torch fp64 autograd."""
    from cvlite import _lib, ops_nn as nn
    if variant == "fallback":
        dispatch("wg_no_x")
    B, C = 4, 256
    shapes = [(24, 20), (12, 10), (6, 5), (3, 3), (2, 2)]
    off, P, xs, dys = _tower_pair_case(B, C, shapes, 21)
    BP = B * P
    w0 = torch.zeros((3, 3, C, C))
    wf = torch.empty((C, 9 * C), dtype=BF, device="cuda")
    wf2 = torch.empty_like(wf)
    segs = []
    for t in range(2):
        src0 = 0 if shared_x else t * BP
        segs += [nn.seg(h, w, h, w, (wf, wf2)[t], None, src_base=src0 + B * off[l], src_img=h * w,
                        dst_base=t * BP + B * off[l], dst_img=h * w) for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, C, C, C, segs)
    dws = [torch.full((3, 3, C, C), 0.25, device="cuda") for _ in range(2)]
    xg, dyg = xs.to(BF).cuda(), dys.to(BF).cuda()
    nn.conv_wgrad_grouped(d, xg, dyg, dws, beta=2.0)
    code = _lib.load().cvl_conv_igemm_last_kernel()
    name = _lib.load().cvl_conv_kernel_name(code).decode()
    print("wgrad kernel:", name)
    if variant == "wx":
        assert code == 11, name
    for t in range(2):
        ref = torch.zeros(3, 3, C, C, dtype=torch.float64)
        for l, (h, w) in enumerate(shapes):
            src0 = 0 if shared_x else t * BP
            xm = xs[src0 + B * off[l]:src0 + B * (off[l] + h * w)].reshape(B, h, w, C)
            wl = w0.double().clone().requires_grad_(True)
            y = ref_conv(xm, wl, None, 1, "same")
            y.backward(dys[t * BP + B * off[l]:t * BP + B * (off[l] + h * w)].reshape(B, h, w, C))
            ref += wl.grad
        exp = ref + 0.5
        scale = ref.abs().max().item()
        torch.testing.assert_close(dws[t].double().cpu(), exp, rtol=1e-4, atol=1e-5 * scale,
                                   msg=lambda m: "tower %d: %s" % (t, m))


def test_conv_wgrad_x_deterministic():
    """The split-M reduction of the 256x256 wgrad kernel sums its fp32 slabs in a fixed order: two
    runs give bit-identical dW (tower-layer shape at bs 16 / 512 for one tower)."""
    from cvlite import _lib, ops_nn as nn
    B, C = 16, 256
    shapes = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    gen = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn((B * P, C), generator=gen, device="cuda").to(BF)
    dy = torch.randn((B * P, C), generator=gen, device="cuda").to(BF)
    wf = torch.empty((C, 9 * C), dtype=BF, device="cuda")
    segs = [nn.seg(h, w, h, w, wf, None, src_base=B * off[l], dst_base=B * off[l]) for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, C, C, C, segs)
    outs = []
    for _ in range(2):
        dw = torch.empty((3, 3, C, C), device="cuda")
        nn.conv_wgrad(d, x, dy, dw)
        assert _lib.load().cvl_conv_igemm_last_kernel() == 11
        outs.append(dw)
    assert torch.equal(outs[0], outs[1])
    # level 0 alone vs torch (fp32 accumulate of the bf16 operands on the GPU)
    xm = x[:B * 4096].float().view(B, 64, 64, C).permute(0, 3, 1, 2)
    dym = dy[:B * 4096].float().view(B, 64, 64, C).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xm.double(), (C, C, 3, 3), dym.double(), padding=1)
    dw0 = torch.empty((3, 3, C, C), device="cuda")
    nn.conv_wgrad(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, C, C, C, segs[:1]), x, dy, dw0)
    torch.testing.assert_close(dw0.double(), ref.permute(2, 3, 1, 0), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("n_store,coff,ld,B,shapes", [
    (20, 0, 32, 3, [(24, 20), (12, 10), (6, 5), (3, 3), (2, 1)]),      # cls head, ragged levels
    (5, 0, 32, 2, [(16, 16), (8, 8), (4, 4), (2, 2), (1, 1)]),          # reg head (t, b, l, r, cen)
    (1, 24, 64, 2, [(9, 7), (5, 4), (3, 2), (2, 1), (1, 1)]),           # centerness column of the cls rows
    (20, 0, 32, 16, [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]),    # bench geometry (bs 16, 512)
])
def test_conv_wgrad_small_n_heads_grouped(n_store, coff, ld, B, shapes):
    """The five per-level FCOS head weight gradients (fcos.py:92-110: 3x3 'same', 256 -> n_store, own
    weights per level) as ONE grouped call (group = level): the small-N kernel conv_wgrad_sn
    (taps on the dY side, deterministic chunk-slab reduction) vs torch fp64 per level, with
    beta accumulation; a second run is bit-identical."""
    from cvlite import _lib, ops_nn as nn
    C = 256
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    g = torch.Generator().manual_seed(7 + n_store)
    x = rnd(B * P, C, gen=g)                                   # packed level-major [sum_l B*h*w, C]
    dy = rnd(B * P, ld, gen=g)                                 # image-major [B, P, ld] loss gradient
    dy[:, coff + n_store:] = 0.0                               # (padding columns are zero in the model)
    wf = [torch.empty((32, 9 * C), dtype=BF, device="cuda") for _ in shapes]
    segs = [nn.seg(h, w, h, w, wf[l], None, src_base=B * off[l], src_img=h * w, dst_base=off[l], dst_img=P)
            for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, 32, n_store, ld, segs, dst_coff=coff)
    xg, dyg = x.to(BF).cuda(), dy.to(BF).cuda()
    outs = []
    for _ in range(2):
        dws = [torch.full((3, 3, C, n_store), 0.5, device="cuda") for _ in shapes]
        nn.conv_wgrad_grouped(d, xg, dyg, dws, beta=1.0)
        code = _lib.load().cvl_conv_igemm_last_kernel()
        assert code == 13, _lib.load().cvl_conv_kernel_name(code).decode()
        outs.append(torch.stack([t.flatten() for t in dws]))
    assert torch.equal(outs[0], outs[1])
    dyi = dy.view(B, P, ld)
    for l, (h, w) in enumerate(shapes):
        xm = x[B * off[l]:B * (off[l] + h * w)].reshape(B, h, w, C)
        ns = max(n_store, 2)                                   # (torch's fp64 CPU conv wants >= 2 outputs)
        dm = torch.zeros(B, h * w, ns, dtype=torch.float64)
        dm[..., :n_store] = dyi[:, off[l]:off[l] + h * w, coff:coff + n_store]
        wl = torch.zeros(3, 3, C, ns, dtype=torch.float64, requires_grad=True)
        ref_conv(xm, wl, None, 1, "same").backward(dm.view(B, h, w, ns))
        exp = wl.grad[..., :n_store] + 0.5
        got = outs[0][l].view(3, 3, C, n_store).double().cpu()
        scale = (exp - 0.5).abs().max().item()
        torch.testing.assert_close(got, exp, rtol=1e-4, atol=1e-5 * scale, msg=lambda m: "level %d: %s" % (l, m))


@pytest.mark.parametrize("B,H,Cin,Cout,k", [(3, 40, 256, 1024, 1), (4, 20, 256, 256, 3), (5, 10, 128, 128, 3),
                                            (2, 40, 256, 256, 3)])
def test_conv_bn_stats_maps_not_tile_aligned(B, H, Cin, Cout, k, kern):
    """Fused BN statistics when H*W % 256 != 0 (RetinaNet 640: 40x40, 20x20 maps; 10x10): a tile's
    waves straddle image boundaries, the per-(wave, image, column) split reduction must equal the
    per-image column sums of the bf16 output."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B * H + Cout)
    x = rnd(B, H, H, Cin, gen=g)
    w = rnd(k, k, Cin, Cout, scale=(k * k * Cin) ** -0.5, gen=g)
    wf, _, npad, _, _ = packs(w)
    bias = (torch.randn(npad, generator=g) * 0.1).float().cuda()
    out = torch.zeros((B, H, H, Cout), dtype=BF, device="cuda")
    stats = nn.bn_acc(B, Cout, "cuda")
    pad = (k - 1) // 2
    d = nn.make_desc(nn.FWD, B, Cin, k, k, 1, pad, pad, npad, Cout, Cout, [nn.seg(H, H, H, H, wf, bias)])
    nn.conv_igemm(d, x.to(BF).cuda(), out, stats)
    o = out.double().cpu()
    st = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
    torch.testing.assert_close(nn.bn_acc_value(stats).cpu(), st, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_conv_wgrad_deferred_reduction():
    """Deferred split reductions (ops_nn.deferred_wgrad, cvl_wgrad_defer / _flush) give dW
    bit-identical to the immediate form: a 1x1 (wgrad_x, 128-wide tiles), a 3x3 (halo kernel) and a
    beta-accumulating second gradient into the SAME dW while the first is still pending (the queue
    flushes before the second record)."""
    from cvlite import ops_nn as nn
    g = torch.Generator(device="cuda").manual_seed(11)
    cases = [(16, 32, 32, 256, 1024, 1), (16, 32, 32, 256, 256, 3)]
    data = []
    for B, H, W, Cin, Cout, k in cases:
        x = torch.randn((B, H, W, Cin), generator=g, device="cuda").to(BF)
        dy = torch.randn((B, H, W, Cout), generator=g, device="cuda").to(BF)
        wf = torch.empty((Cout, k * k * Cin), dtype=BF, device="cuda")
        d = nn.make_desc(nn.FWD, B, Cin, k, k, 1, k // 2, k // 2, Cout, Cout, Cout, [nn.seg(H, W, H, W, wf)])
        data.append((d, x, dy, (k, k, Cin, Cout)))

    def run(deferred):
        outs = [torch.zeros(s, device="cuda") for (_, _, _, s) in data]
        acc = torch.ones(data[0][3], device="cuda")

        def body():
            for (d, x, dy, _), o in zip(data, outs):
                nn.conv_wgrad(d, x, dy, o)
            nn.conv_wgrad(data[0][0], data[0][1], data[0][2], acc, beta=0.5)
            nn.conv_wgrad(data[0][0], data[0][1], data[0][2], acc, beta=1.0)   # same dW, first still pending
        if deferred:
            with nn.deferred_wgrad():
                body()
                nn.wgrad_flush()
        else:
            body()
        torch.cuda.synchronize()
        return outs + [acc]

    imm, dfr = run(False), run(True)
    for a, b in zip(imm, dfr):
        assert torch.equal(a, b)
    # and the accumulated one is 0.5 + 2 * dW (fp32 tolerance)
    torch.testing.assert_close(imm[2], 0.5 + 2 * imm[0], rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_conv_wgrad_deferred_then_direct_writer():
    """a dW whose split reduction is still pending (deferral on, beta 0) is then
    accumulated (beta 1) by a launch on a DIRECT-writing path (the small-N head kernel, no slabs):
    cvl_conv_wgrad_grouped flushes the pending record before any path writes, so the result is
    bit-identical to the immediate form (without the guard the late reduction overwrote the
    direct write)."""
    from cvlite import _lib, ops_nn as nn
    g = torch.Generator(device="cuda").manual_seed(5)
    B, H, W, Cin, Cout = 16, 32, 32, 256, 1024
    x1 = torch.randn((B, H, W, Cin), generator=g, device="cuda").to(BF)
    dy1 = torch.randn((B, H, W, Cout), generator=g, device="cuda").to(BF)
    wf1 = torch.empty((Cout, Cin), dtype=BF, device="cuda")
    d1 = nn.make_desc(nn.FWD, B, Cin, 1, 1, 1, 0, 0, Cout, Cout, Cout, [nn.seg(H, W, H, W, wf1)])
    B2, H2, n2 = 2, 16, 20
    x2 = torch.randn((B2, H2, H2, Cin), generator=g, device="cuda").to(BF)
    dy2 = torch.randn((B2, H2, H2, 32), generator=g, device="cuda").to(BF)
    wf2 = torch.empty((32, 9 * Cin), dtype=BF, device="cuda")
    d2 = nn.make_desc(nn.FWD, B2, Cin, 3, 3, 1, 1, 1, 32, n2, 32, [nn.seg(H2, H2, H2, H2, wf2)])
    kinds = []

    def run(deferred):
        dw = torch.zeros((Cin, Cout), device="cuda")
        head = dw.view(-1)[:9 * Cin * n2].view(3, 3, Cin, n2)        # same base pointer as dw

        def body():
            nn.conv_wgrad(d1, x1, dy1, dw)
            kinds.append(int(_lib.load().cvl_conv_igemm_last_kernel()))
            nn.conv_wgrad(d2, x2, dy2, head, beta=1.0)
            kinds.append(int(_lib.load().cvl_conv_igemm_last_kernel()))
        if deferred:
            with nn.deferred_wgrad():
                body()
                nn.wgrad_flush()
        else:
            body()
        torch.cuda.synchronize()
        return dw

    imm, dfr = run(False), run(True)
    assert kinds[0] == 11 and kinds[1] != 11, kinds        # split wgrad_x first, a non-split writer second
    assert torch.equal(imm, dfr)


@pytest.mark.parametrize("case", [(16, 16, 2048, 256), (16, 8, 256, 256), (3, 12, 64, 96)])
def test_s2_3x3_dgrad_parity_form(dispatch, case):
    """3x3 stride-2 data gradient on even maps (TF 'same', zero leading pad: the FPN P6 / P7 convs)
    through the 4-segment parity form (2x2 sub-kernels gathered from the dgrad pack, dst_up = 2
    scatter) vs the direct 9-tap form (CVL_DISPATCH=no_s2dg3) and fp64 autograd; into a wider
    destination at a channel offset with beta = 1 as well (s2dg3_min_rows=1: the small maps too)."""
    import ctypes
    from cvlite import _lib, ops_nn as nn
    B, H, Cin, Cout = case
    dispatch("s2dg3_min_rows=1")
    g = torch.Generator().manual_seed(H * 7 + Cin)
    x = rnd(B, H, H, Cin, gen=g).cuda().requires_grad_(True)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g).cuda().requires_grad_(True)
    xn = x.permute(0, 3, 1, 2)
    y = F.conv2d(F.pad(xn, (0, 1, 0, 1)), w.permute(3, 2, 0, 1), None, 2).permute(0, 2, 3, 1)
    Ho = y.shape[1]
    dy = rnd(*y.shape, gen=g).cuda()
    y.backward(dy)
    _, wd, _, cout_pad, cin_pad = packs(w.detach().cpu())
    dyg = torch.zeros((B, Ho, Ho, cout_pad), dtype=BF, device="cuda")
    dyg[..., :Cout] = dy.to(BF)
    ld = Cin + 16
    old = torch.randn((B, H, H, ld), generator=g).to(BF).cuda()
    outs = []
    for off in ("0", "1"):
        dispatch("no_s2dg3=" + off)
        d = nn.make_desc(nn.DGRAD, B, cout_pad, 3, 3, 2, 0, 0, cin_pad, Cin, Cin, [nn.seg(H, H, Ho, Ho, wd)])
        if off == "0":
            assert _lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(d)) >= 16 * cin_pad * cout_pad * 2
        dx = torch.empty((B, H, H, Cin), dtype=BF, device="cuda")
        nn.conv_igemm(d, dyg, dx)
        d2 = nn.make_desc(nn.DGRAD, B, cout_pad, 3, 3, 2, 0, 0, cin_pad, Cin, ld, [nn.seg(H, H, Ho, Ho, wd)],
                          dst_coff=8, beta=1.0)
        dx2 = old.clone()
        nn.conv_igemm(d2, dyg, dx2)
        outs.append((dx.double(), dx2.double()))
    for dx, dx2 in outs:
        torch.testing.assert_close(dx, x.grad, rtol=1e-2, atol=2e-2)
        exp = old.double().clone()
        exp[..., 8:8 + Cin] += x.grad
        torch.testing.assert_close(dx2, exp, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,H", [(4, 64), (3, 20)])
def test_head_dgrad_cin32_on_x32(dispatch, B, H):
    """The heads' data gradient (3x3, 32 gradient channels -> 256, K = 288) on the X32 ring kernel
    (CVL_DISPATCH=x_cin32) and on the default path, both against fp64 autograd."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B * 100 + H)
    Cin, Cout = 256, 32
    x = rnd(B, H, H, Cin, gen=g).cuda().requires_grad_(True)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g).cuda().requires_grad_(True)
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), None, 1, 1).permute(0, 2, 3, 1)
    dy = rnd(*y.shape, gen=g).cuda()
    y.backward(dy)
    _, wd, _, cout_pad, cin_pad = packs(w.detach().cpu())
    dyg = dy.to(BF).contiguous()
    outs = []
    for on in ("1", "0"):
        dispatch("x_cin32=" + on)
        dx = torch.empty((B, H, H, Cin), dtype=BF, device="cuda")
        d = nn.make_desc(nn.DGRAD, B, cout_pad, 3, 3, 1, 1, 1, cin_pad, Cin, Cin, [nn.seg(H, H, H, H, wd)])
        nn.conv_igemm(d, dyg, dx)
        if on == "1":
            from cvlite import _lib
            assert _lib.load().cvl_conv_igemm_last_kernel() == 7
        outs.append(dx.double())
    for o in outs:
        torch.testing.assert_close(o, x.grad, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("fuse", [True, False], ids=["epilogue", "fallback"])
def test_conv_igemm_relu_mask_matches_dgrad_then_relu(dispatch, fuse):
    """cvl_conv_igemm_relu_mask (the FCOS heads' data gradients into the towers' final ReLU output,
    fcos.py:16-27 / 76-101): bit-identical to cvl_conv_igemm + cvl_relu_backward, through the tower
    kernel's register epilogue (bench geometry: the five levels at bs 16) and through the fallback
    (CVL_DISPATCH=no_relu_mask_fuse: the plain launch, then the separate ReLU backward)."""
    from cvlite import _lib, ops_nn as nn
    if not fuse:
        dispatch("no_relu_mask_fuse")
    B, C, NS = 16, 256, 32
    shapes = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    P = o
    g = torch.Generator().manual_seed(31)
    dout = rnd(B * P, NS, gen=g).to(BF).cuda()                     # head gradients [B, P, 32] image-major
    y = torch.relu(rnd(B * P, C, gen=g)).to(BF).cuda()             # tower ReLU output, level-major
    y[::7, ::3] = 0.0
    wd = [rnd(C, 9 * NS, scale=0.05, gen=g).to(BF).cuda() for _ in shapes]
    segs = [nn.seg(h, w, h, w, wd[l], None, src_base=off[l], src_img=P, dst_base=B * off[l], dst_img=h * w)
            for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.DGRAD, B, NS, 3, 3, 1, 1, 1, C, C, C, segs)
    ref = torch.empty((B * P, C), dtype=BF, device="cuda")
    nn.conv_igemm(d, dout, ref)
    nn.relu_backward(ref, y, ref)
    got = torch.full((B * P, C), 3.0, dtype=BF, device="cuda")
    nn.conv_igemm_relu_mask(d, dout, got, y)
    name = _lib.load().cvl_conv_kernel_name(_lib.load().cvl_conv_igemm_last_kernel()).decode()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), name
    assert float(got[y == 0].abs().max()) == 0.0
