"""The halo-staged 256 x 64 conv kernel (conv_igemm_h.hip, CVL_CK_H64): 3x3 / stride 1 launches of
the ResNet-50 3x3 units, the FPN output convs and narrow tower launches (Keras ResNet50 behind
FCOS/fcos.py:30-46; fcos.py:62-66) -- forward and data gradient on every map geometry it takes
(whole image rows at W = 128 .. 16, mosaics of whole small images at 8x8 / 4x4, several segments
in one launch), with bias / ReLU / BN statistics / beta / fp32 destinations, the split-K form for
small grids, and the fused BN-backward first pass; vs a float64 convolution of the same bf16
operands (bf16 outputs: one rounding, rtol/atol 1e-2; fp32 outputs 1e-4)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rnd(*shape, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen, dtype=torch.float64) * scale).to(BF).to(torch.float64)


def conv3(x, w, b=None):
    """x NHWC, w HWIO float64, TF 'same' 3x3 stride 1."""
    return F.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b, 1, 1).permute(0, 2, 3, 1)


def packs(w):
    from cvlite import ops_nn as nn
    k, _, cin, cout = w.shape
    npad = (cout + 31) // 32 * 32
    cin_pad = (cin + 31) // 32 * 32
    wf = torch.empty((npad, k * k * cin), dtype=BF, device="cuda")
    wd = torch.empty((cin_pad, k * k * npad), dtype=BF, device="cuda")
    nn.pack_conv_weights(w.float().cuda().contiguous(), k, k, cin, cout, cin, npad, wf, cin_pad, npad, wd)
    return wf, wd, npad, cin_pad


def last_kernel():
    from cvlite import _lib
    L = _lib.load()
    return L.cvl_conv_kernel_name(L.cvl_conv_igemm_last_kernel()).decode()


CASES = [  # (B, H, W, Cin, Cout): conv2_x..conv5_x 3x3 units at reduced batch, odd channel counts
    (2, 128, 128, 64, 64),
    (3, 64, 64, 128, 128),
    (4, 32, 32, 256, 192),
    (8, 16, 16, 512, 64),
    (5, 8, 8, 32, 64),
    (3, 4, 4, 64, 128),
]


@pytest.mark.parametrize("case", CASES)
def test_h_fwd_dgrad(case):
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout = case
    g = torch.Generator().manual_seed(B * 1000 + H + Cin + Cout)
    x = rnd(B, H, W, Cin, gen=g).requires_grad_(True)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    wf, wd, npad, cin_pad = packs(w)
    bias = b.float().cuda()
    xg = x.detach().to(BF).cuda()
    # forward: bias + ReLU + BN statistics (bf16), then fp32 into a wider buffer with beta = 1
    ref = conv3(x.detach(), w, b).clamp(min=0)
    out = torch.zeros((B, H, W, Cout), dtype=BF, device="cuda")
    st = nn.bn_acc(B, Cout, "cuda")
    d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, Cout, [nn.seg(H, W, H, W, wf, bias)], relu_out=True)
    nn.conv_igemm(d, xg, out, st)
    assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-2, atol=1e-2)
    o = out.double().cpu()
    torch.testing.assert_close(nn.bn_acc_value(st).cpu(), torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1), rtol=1e-5,
                               atol=1e-3)
    ld = Cout + 8
    o32 = torch.randn((B, H, W, ld), generator=g).cuda()
    before = o32.clone()
    d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, ld, [nn.seg(H, W, H, W, wf, bias)], dst_coff=8,
                     dst_f32=True, beta=1.0)
    nn.conv_igemm(d, xg, o32)
    exp = before.double().cpu()
    exp[..., 8:8 + Cout] += conv3(x.detach(), w, b)
    torch.testing.assert_close(o32.double().cpu(), exp, rtol=1e-4, atol=1e-4)
    # data gradient (dgrad pack), then beta = 1 accumulation
    y = conv3(x, w)
    dy = rnd(*y.shape, gen=g)
    y.backward(dy)
    dyg = torch.zeros((B, H, W, npad), dtype=BF, device="cuda")
    dyg[..., :Cout] = dy.to(BF).cuda()
    if cin_pad % 64:
        return                      # dgrad Npad = Cin_pad: the kernel takes multiples of 64
    dx = torch.empty((B, H, W, Cin), dtype=BF, device="cuda")
    dd = nn.make_desc(nn.DGRAD, B, npad, 3, 3, 1, 1, 1, cin_pad, Cin, Cin, [nn.seg(H, W, H, W, wd)])
    nn.conv_igemm(dd, dyg, dx)
    assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
    torch.testing.assert_close(dx.double().cpu(), x.grad, rtol=1e-2, atol=2e-2)
    old = torch.randn((B, H, W, Cin), generator=g).to(BF)
    dx2 = old.cuda()
    dd = nn.make_desc(nn.DGRAD, B, npad, 3, 3, 1, 1, 1, cin_pad, Cin, Cin, [nn.seg(H, W, H, W, wd)], beta=1.0)
    nn.conv_igemm(dd, dyg, dx2)
    torch.testing.assert_close(dx2.double().cpu(), x.grad + old.double(), rtol=1e-2, atol=3e-2)


@pytest.mark.parametrize("B,H,Cin", [(4, 128, 64), (3, 8, 32), (16, 128, 64)])
def test_h_resident_weights_bit_identical(B, H, Cin, dispatch):
    """WRES (weights resident in LDS for single-N-tile launches with Cin <= 64: the conv2_x 3x3 units,
    halos streamed alone) gives the same bits as the per-block weight staging (CVL_DISPATCH=h_no_wres):
    forward with bias / ReLU / BN statistics, data gradient, and the data gradient with the fused
    BN-backward first pass (the step's form), including the bs 16 128x128 geometry."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B + H + Cin)
    Cout = 64
    x = rnd(B, H, H, Cin, gen=g)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g)
    wf, wd, npad, cin_pad = packs(w)
    bias = torch.randn(Cout, generator=g).cuda()
    xg = x.to(BF).cuda()
    dy = rnd(B, H, H, Cout, gen=g).to(BF).cuda()
    z = rnd(B, H, H, Cin, gen=g).to(BF).cuda()
    mr = torch.stack([torch.randn(B, Cin, generator=g) * 0.2, torch.rand(B, Cin, generator=g) + 0.5], -1).cuda()
    ga, be = (torch.rand(Cin, generator=g) + 0.5).cuda(), torch.randn(Cin, generator=g).cuda()
    res = []
    for off in ("1", "0"):
        dispatch("h_no_wres=" + off)
        out = torch.empty((B, H, H, Cout), dtype=BF, device="cuda")
        st = nn.bn_acc(B, Cout, "cuda")
        d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, Cout, [nn.seg(H, H, H, H, wf, bias)], relu_out=True)
        nn.conv_igemm(d, xg, out, st)
        k_fwd = last_kernel()
        dx = torch.empty((B, H, H, Cin), dtype=BF, device="cuda")
        dd = nn.make_desc(nn.DGRAD, B, npad, 3, 3, 1, 1, 1, cin_pad, Cin, Cin, [nn.seg(H, H, H, H, wd)])
        nn.conv_igemm(dd, dy, dx)
        dx2 = torch.empty_like(dx)
        sums = nn.bn_acc(B, Cin, "cuda")
        fused = nn.conv_igemm_dgrad_bnsum(dd, dy, dx2, z, mr, ga, be, sums)
        torch.cuda.synchronize()
        res.append((out.view(torch.int16), dx.view(torch.int16), dx2.view(torch.int16), nn.bn_acc_value(st),
                    nn.bn_acc_value(sums) if fused else None, k_fwd))
    a, b2 = res
    assert "conv_igemm_h_kernel" in a[5] and "conv_igemm_h_kernel" in b2[5]
    for u, v in zip(a[:3], b2[:3]):
        assert torch.equal(u, v)
    torch.testing.assert_close(a[3], b2[3], rtol=1e-12, atol=1e-9)
    if a[4] is not None:
        torch.testing.assert_close(a[4], b2[4], rtol=1e-12, atol=1e-9 * float(a[4].abs().max()))


@pytest.mark.parametrize("B,H,Cin,Cout", [(16, 128, 64, 64), (4, 64, 128, 128), (4, 32, 256, 256), (2, 16, 512, 512),
                                          (3, 8, 32, 64)])
def test_h_register_epilogue_matches_c_image(B, H, Cin, Cout, dispatch):
    """The SW epilogue (swapped MFMA operands, 16-B stores straight from registers, BN statistics /
    BN-backward sums kept per (image, N tile) and flushed once per change) against the LDS C-image
    epilogue (CVL_DISPATCH=h_no_sw): forward with bias / ReLU / BN statistics, data gradient, data
    gradient with the fused BN-backward first pass, at the backbone 3x3 geometries (conv2_x..conv5_x,
    bs 16 / 4 / 2: one or several tiles and N tiles per workgroup) and a mosaic map (8x8: SW does
    not apply, both runs take the C-image form).  Outputs bit-identical (the MFMA forms the same dot
    products); the sums differ only in fp32 summation order."""
    from cvlite import ops_nn as nn
    g = torch.Generator().manual_seed(B * 7 + H + Cin)
    x = rnd(B, H, H, Cin, gen=g)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g)
    wf, wd, npad, cin_pad = packs(w)
    bias = torch.randn(Cout, generator=g).cuda()
    xg = x.to(BF).cuda()
    dy = rnd(B, H, H, Cout, gen=g).to(BF).cuda()
    z = rnd(B, H, H, Cin, gen=g).to(BF).cuda()
    mr = torch.stack([torch.randn(B, Cin, generator=g) * 0.2, torch.rand(B, Cin, generator=g) + 0.5], -1).cuda()
    ga, be = (torch.rand(Cin, generator=g) + 0.5).cuda(), torch.randn(Cin, generator=g).cuda()
    res = []
    for off in ("1", "0"):
        dispatch("h_no_sw=" + off)
        out = torch.empty((B, H, H, Cout), dtype=BF, device="cuda")
        st = nn.bn_acc(B, Cout, "cuda")
        d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, Cout, [nn.seg(H, H, H, H, wf, bias)], relu_out=True)
        nn.conv_igemm(d, xg, out, st)
        k_fwd = last_kernel()
        dx = torch.empty((B, H, H, Cin), dtype=BF, device="cuda")
        dd = nn.make_desc(nn.DGRAD, B, npad, 3, 3, 1, 1, 1, cin_pad, Cin, Cin, [nn.seg(H, H, H, H, wd)])
        nn.conv_igemm(dd, dy, dx)
        dx2 = torch.empty_like(dx)
        sums = nn.bn_acc(B, Cin, "cuda")
        fused = nn.conv_igemm_dgrad_bnsum(dd, dy, dx2, z, mr, ga, be, sums)
        torch.cuda.synchronize()
        res.append((out.view(torch.int16), dx.view(torch.int16), dx2.view(torch.int16), nn.bn_acc_value(st),
                    nn.bn_acc_value(sums) if fused else None, k_fwd))
    a, b2 = res
    assert "conv_igemm_h_kernel" in a[5] and "conv_igemm_h_kernel" in b2[5], (a[5], b2[5])
    for name, u, v in zip(("fwd", "dgrad", "dgrad+bnsum"), a[:3], b2[:3]):
        assert torch.equal(u, v), name
    torch.testing.assert_close(a[3], b2[3], rtol=2e-5, atol=1e-3)
    if a[4] is not None:
        torch.testing.assert_close(a[4], b2[4], rtol=2e-5, atol=2e-5 * float(a[4].abs().max()))


def test_h_segments_fpn_trio(dispatch):
    """The FPN's three 3x3 output convs (fcos.py:62-66: P3r, P4r, P5 -> P3, P4, P5, own weights and
    biases) as ONE 3-segment launch from one packed source buffer into the level-major F buffer."""
    from cvlite import ops_nn as nn
    B, C = 2, 256
    shapes = [(64, 64), (32, 32), (16, 16)]
    g = torch.Generator().manual_seed(11)
    maps = [rnd(B, h, w, C, gen=g) for h, w in shapes]
    src = torch.cat([m.reshape(-1, C) for m in maps], 0).to(BF).cuda()
    ws = [rnd(3, 3, C, C, scale=(9 * C) ** -0.5, gen=g) for _ in shapes]
    bs = [torch.randn(C, generator=g, dtype=torch.float64) for _ in shapes]
    pk = [packs(w) for w in ws]
    base, o = [], 0
    for h, w in shapes:
        base.append(o)
        o += B * h * w
    segs = [nn.seg(h, w, h, w, pk[l][0], bs[l].float().cuda(), src_base=base[l], dst_base=base[l])
            for l, (h, w) in enumerate(shapes)]
    out = torch.empty_like(src)
    # 256-wide tiles would go to the 256 x 256 kernels; force the narrow path for the trio
    dispatch("no_256")
    nn.conv_igemm(nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, C, C, C, segs), src, out)
    assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
    for l, (h, w) in enumerate(shapes):
        got = out[base[l]:base[l] + B * h * w].reshape(B, h, w, C).double().cpu()
        torch.testing.assert_close(got, conv3(maps[l], ws[l], bs[l]), rtol=1e-2, atol=1e-2)


def test_h_split_k_small_grid():
    """conv5_x 3x3 (512 -> 512 @ 16x16) at bs 4: 16 x 8 = 128 tiles split over channel blocks
    (fp32 slabs + finishing pass with bias / ReLU / BN statistics) == the unsplit launch."""
    import ctypes
    from cvlite import _lib, ops_nn as nn
    B, H, Cin, Cout = 16, 16, 512, 512
    g = torch.Generator().manual_seed(5)
    x = rnd(B, H, H, Cin, gen=g)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    wf, _, npad, _ = packs(w)
    d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, Cout, [nn.seg(H, H, H, H, wf, b.float().cuda())],
                     relu_out=True)
    n = int(_lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(d)))
    assert n > 16
    outs, sts = [], []
    for split in (True, False):
        out = torch.zeros((B, H, H, Cout), dtype=BF, device="cuda")
        st = nn.bn_acc(B, Cout, "cuda")
        if split:
            nn.conv_igemm(d, x.to(BF).cuda(), out, st)
        else:
            _lib.call("cvl_conv_igemm", ctypes.byref(d), _lib.ptr(x.to(BF).cuda()), _lib.ptr(out), _lib.ptr(st),
                      None, 0, _lib.stream())
        assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
        outs.append(out.double().cpu())
        sts.append(nn.bn_acc_value(st).cpu())
    ref = conv3(x, w, b).clamp(min=0)
    for o, st in zip(outs, sts):
        torch.testing.assert_close(o, ref, rtol=1e-2, atol=1e-2)
        # each path's statistics are those of its own output (to the bf16 rounding of the stored values)
        torch.testing.assert_close(st, torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-2, atol=1e-2)


def test_h_32_wide_tiles_conv5(dispatch):
    """conv5_x 3x3 (512 -> 512 @ 16x16, bs 16: 128 tiles of 256 x 64) on 256 x 32 tiles (round 6:
    every CU a tile, no split-K slabs): forward with bias / ReLU / BN statistics vs float64, the data
    gradient with the fused BN-backward first pass bit-identical to the 64-wide launch (same MFMA dot
    products; the sums to fp32 order)."""
    from cvlite import ops_nn as nn
    B, H, C = 16, 16, 512
    g = torch.Generator().manual_seed(21)
    x = rnd(B, H, H, C, gen=g)
    w = rnd(3, 3, C, C, scale=(9 * C) ** -0.5, gen=g)
    b = torch.randn(C, generator=g, dtype=torch.float64)
    wf, wd, npad, cin_pad = packs(w)
    xg = x.to(BF).cuda()
    dy = rnd(B, H, H, C, gen=g).to(BF).cuda()
    z = rnd(B, H, H, C, gen=g).to(BF).cuda()
    mr = torch.stack([torch.randn(B, C, generator=g) * 0.2, torch.rand(B, C, generator=g) + 0.5], -1).cuda()
    ga, be = (torch.rand(C, generator=g) + 0.5).cuda(), torch.randn(C, generator=g).cuda()
    out = torch.empty((B, H, H, C), dtype=BF, device="cuda")
    st = nn.bn_acc(B, C, "cuda")
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, npad, C, C, [nn.seg(H, H, H, H, wf, b.float().cuda())], relu_out=True)
    nn.conv_igemm(d, xg, out, st)
    assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
    o = out.double().cpu()
    torch.testing.assert_close(o, conv3(x, w, b).clamp(min=0), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(nn.bn_acc_value(st).cpu(), torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1),
                               rtol=1e-4, atol=1e-2)
    dd = nn.make_desc(nn.DGRAD, B, npad, 3, 3, 1, 1, 1, cin_pad, C, C, [nn.seg(H, H, H, H, wd)])
    res = []
    for off in ("0", "1"):
        dispatch("h_no_n32=" + off)
        dx = torch.empty((B, H, H, C), dtype=BF, device="cuda")
        sums = nn.bn_acc(B, C, "cuda")
        assert nn.conv_igemm_dgrad_bnsum(dd, dy, dx, z, mr, ga, be, sums)
        assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
        res.append((dx.view(torch.int16), nn.bn_acc_value(sums)))
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=2e-5, atol=2e-5 * float(res[1][1].abs().max()))


def test_h_dgrad_fused_bn_backward_sums():
    """conv2_x's 3x3 data gradient with the conv1 unit's BN-backward first pass in the epilogue
    (cvl_conv_igemm_dgrad_bnsum on H64): dX identical to the plain launch, sums vs float64."""
    from cvlite import ops_nn as nn
    from cvlite.layers import Conv, ParamStore
    B, H, C = 2, 128, 64
    dev = torch.device("cuda")
    st = ParamStore()
    conv = Conv(st, "c", 3, C, C, 1, "same", bias=False)
    st.finalize(dev, seed=3)
    conv.pack()
    g = torch.Generator().manual_seed(9)
    dy_next = (torch.randn(B, H, H, C, generator=g) * 0.5).to(BF).to(dev)
    z = (torch.randn(B, H, H, C, generator=g) * 1.5 + 0.2).to(BF).to(dev)
    mr = torch.empty((B, C, 2), dtype=torch.float32, device=dev)
    zf = z.double().view(B, H * H, C)
    mr[..., 0] = zf.mean(1).float()
    mr[..., 1] = torch.rsqrt(zf.var(1, unbiased=False) + 1e-3).float()
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = torch.randn(C, generator=g).to(dev) * 0.3
    d = conv.dgrad_desc(B, [nn.seg(H, H, H, H, conv.wd)], ld_dst=C)
    dx_f = torch.empty((B, H, H, C), dtype=BF, device=dev)
    sums = nn.bn_acc(B, C, dev)
    assert nn.conv_igemm_dgrad_bnsum(d, dy_next, dx_f, z, mr, gamma, beta, sums)
    assert "conv_igemm_h_kernel" in last_kernel(), last_kernel()
    dx_p = torch.empty_like(dx_f)
    nn.conv_igemm(d, dy_next, dx_p)
    assert torch.equal(dx_f, dx_p)
    xh = (z.float() - mr[..., 0].view(B, 1, 1, C)) * mr[..., 1].view(B, 1, 1, C)
    a = gamma * xh + beta
    gm = torch.where(a > 0, dx_p.float(), torch.zeros_like(a)).double()
    ref = torch.stack([gm.sum((1, 2)), (gm * xh.double()).sum((1, 2))], -1)
    torch.testing.assert_close(nn.bn_acc_value(sums), ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))


WG_CASES = [  # (B, H, W, Cin, Cout): the 3x3 units' weight gradients (conv2_x..conv5_x), FPN c4/c5
    (2, 128, 128, 64, 64),
    (2, 64, 64, 128, 128),
    (4, 32, 32, 256, 256),
    (16, 16, 16, 512, 512),
    (1, 16, 16, 64, 128),
]


@pytest.mark.parametrize("case", WG_CASES)
def test_h_wgrad(case):
    """conv_wgrad_h_kernel (halo-staged 3x3 weight gradient, split over row chunks with a
    fixed-order slab reduction, or direct with beta) vs float64 on the same bf16 operands."""
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout = case
    g = torch.Generator().manual_seed(H * Cin + Cout + B)
    x = rnd(B, H, W, Cin, gen=g)
    w = rnd(3, 3, Cin, Cout, scale=(9 * Cin) ** -0.5, gen=g).requires_grad_(True)
    y = conv3(x, w)
    dy = rnd(*y.shape, gen=g)
    y.backward(dy)
    wf, _, npad, _ = packs(w.detach())
    ld = Cout + 8                                     # dY rows wider than Cout, at a channel offset
    dyg = torch.zeros((B, H, W, ld), dtype=BF, device="cuda")
    dyg[..., 8:8 + Cout] = dy.to(BF).cuda()
    d = nn.make_desc(nn.FWD, B, Cin, 3, 3, 1, 1, 1, npad, Cout, ld, [nn.seg(H, W, H, W, wf)], dst_coff=8)
    old = torch.randn((3, 3, Cin, Cout), generator=g).cuda()
    dw = old.clone()
    nn.conv_wgrad(d, x.to(BF).cuda(), dyg, dw, beta=1.0)
    assert "conv_wgrad_h_kernel" in last_kernel(), last_kernel()
    ref = w.grad + old.double().cpu()
    scale = float(w.grad.abs().max())
    torch.testing.assert_close(dw.double().cpu(), ref, rtol=1e-4, atol=2e-5 * scale)
    dw0 = torch.zeros((3, 3, Cin, Cout), device="cuda")
    nn.conv_wgrad(d, x.to(BF).cuda(), dyg, dw0)
    torch.testing.assert_close(dw0.double().cpu(), w.grad, rtol=1e-4, atol=2e-5 * scale)
