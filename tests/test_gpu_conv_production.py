"""GPU parity of the conv launches that carry the FCOS / RetinaNet step at BASELINE sizes, through
the kernel the production dispatch picks (no dispatch knobs): the paired cls+reg tower layer
(FCOS/fcos.py:16-27, 76-101; 10 segments = 2 towers x 5 FPN levels, Cin = Npad = 256) at the
configs[1] layout (bs 16, 512x512: M = 174,592 rows), forward and data gradient; a 256-wide
1x1 backbone conv with fused BN statistics (conv2_x expand at bs 16); the fp32-destination
epilogue of the RetinaNet grouped class head (retinanet_module.py:107-148, C = 80: Npad 768,
n_store 720) at configs[4] (bs 8, 640x640) and that head's data gradient.

Reference: the same convolution in float64 on the GPU (nine shifted-view matmuls on the same
bf16-rounded operands), i.e. independent of every cvlite kernel.  Tolerances (stated here as in
tests/test_gpu_conv.py): bf16 outputs rtol/atol 1e-2 (one bf16 rounding of the result), fp32
outputs 1e-4, BN statistics rtol 1e-5 of the sums of the bf16 outputs."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F64 = torch.float64


def last_kernel():
    from cvlite import _lib
    lib = _lib.load()
    code = lib.cvl_conv_igemm_last_kernel()
    return code, lib.cvl_conv_kernel_name(code).decode()


def conv_ref(x, w, stride=1, pt=1, pl=1, Ho=None, Wo=None):
    """x [B,H,W,C] fp64 cuda, w HWIO fp64 cuda -> [B,Ho,Wo,N] fp64 (zero padding pt/pl)."""
    B, H, W, C = x.shape
    k = w.shape[0]
    Ho = Ho or (H + stride - 1) // stride
    Wo = Wo or (W + stride - 1) // stride
    xp = torch.nn.functional.pad(x, (0, 0, pl, k, pt, k))
    out = torch.zeros((B, Ho, Wo, w.shape[3]), dtype=F64, device=x.device)
    for r in range(k):
        for s in range(k):
            patch = xp[:, r:r + stride * (Ho - 1) + 1:stride, s:s + stride * (Wo - 1) + 1:stride, :]
            out += torch.matmul(patch, w[r, s])
    return out


def dgrad_ref(dy, w):
    """3x3 stride-1 'same' data gradient = 'same' conv of dy with the flipped, transposed kernel."""
    return conv_ref(dy, w.flip(0).flip(1).transpose(2, 3).contiguous())


def packs(w, npad=None, cout_pad=None):
    from cvlite import ops_nn as nn
    k, _, cin, cout = w.shape
    npad = npad or max(32, (cout + 31) // 32 * 32)
    cout_pad = cout_pad or npad
    cin_pad = (cin + 31) // 32 * 32
    wf = torch.empty((npad, k * k * cin), dtype=BF, device="cuda")
    wd = torch.empty((cin_pad, k * k * cout_pad), dtype=BF, device="cuda")
    nn.pack_conv_weights(w.float().contiguous(), k, k, cin, cout, cin, npad, wf, cin_pad, cout_pad, wd)
    return wf, wd


def rnd(shape, scale, gen):
    return (torch.randn(shape, generator=gen, device="cuda", dtype=torch.float32) * scale).to(BF)


def fpn_layout(B, S):
    shapes = [(-(-S // s), -(-S // s)) for s in (8, 16, 32, 64, 128)]
    off, o = [], 0
    for h, w in shapes:
        off.append(o)
        o += h * w
    return shapes, off, o


def test_tower_pair_fwd_dgrad_configs1_layout():
    """One paired tower layer exactly as FPNDetector._pair_segs lays it out at bs 16 / 512."""
    from cvlite import ops_nn as nn
    B, S, C = 16, 512, 256
    shapes, off, P = fpn_layout(B, S)
    BP = B * P
    g = torch.Generator(device="cuda").manual_seed(11)
    src = rnd((2 * BP, C), 0.5, g)
    ws = [rnd((3, 3, C, C), (9 * C) ** -0.5, g).to(F64) for _ in range(2)]
    pk = [packs(w) for w in ws]
    segs = []
    for t in range(2):
        segs += [nn.seg(h, w, h, w, pk[t][0], None, src_base=t * BP + B * off[l], src_img=h * w,
                        dst_base=t * BP + B * off[l], dst_img=h * w) for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, C, C, C, segs)
    out = torch.empty_like(src)
    nn.conv_igemm(d, src, out)
    code, name = last_kernel()
    print("forward kernel:", name)
    assert code == 7, name                  # X32: the 256x256 LDS-DMA tile the bench's roofline names
    srcd = src.to(F64)
    for t in range(2):
        for l, (h, w) in enumerate(shapes):
            r0 = t * BP + B * off[l]
            x = srcd[r0:r0 + B * h * w].view(B, h, w, C)
            ref = conv_ref(x, ws[t])
            got = out[r0:r0 + B * h * w].view(B, h, w, C).to(F64)
            torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2, msg=lambda m: "tower %d level %d: %s" % (t, l, m))
    # data gradient: both towers' layer in ONE 10-segment launch over the paired gradient buffer
    dsegs = []
    for t in range(2):
        dsegs += [nn.seg(h, w, h, w, pk[t][1], None, src_base=t * BP + B * off[l], src_img=h * w,
                         dst_base=t * BP + B * off[l], dst_img=h * w) for l, (h, w) in enumerate(shapes)]
    dd = nn.make_desc(nn.DGRAD, B, C, 3, 3, 1, 1, 1, C, C, C, dsegs)
    dy = rnd((2 * BP, C), 1.0, g)
    dx = torch.empty_like(dy)
    nn.conv_igemm(dd, dy, dx)
    code, name = last_kernel()
    print("dgrad kernel:", name)
    assert code == 7, name
    dyd = dy.to(F64)
    for t in range(2):
        for l, (h, w) in enumerate(shapes):
            r0 = t * BP + B * off[l]
            ref = dgrad_ref(dyd[r0:r0 + B * h * w].view(B, h, w, C), ws[t])
            got = dx[r0:r0 + B * h * w].view(B, h, w, C).to(F64)
            torch.testing.assert_close(got, ref, rtol=1e-2, atol=2e-2, msg=lambda m: "dgrad tower %d level %d: %s" % (t, l, m))


@pytest.mark.parametrize("variant", ["p", "p64", "p256", "l128", "wide"])
def test_wide_1x1_with_bn_stats_configs1(variant, dispatch):
    """conv2_block1_3 (1x1 64 -> 256 at 128x128, bs 16: 1,024 M tiles) with the fused per-image BN
    statistics epilogue, as ConvBN.forward runs it: on the persistent 1x1 kernel (default; also
    forced to its 64- and 256-wide tiles), and with it off on the one-tile-per-workgroup L kernel's
    256x128 tile and forced onto the 256-wide tiles (CVL_DISPATCH=w256_min_k=0)."""
    from cvlite import ops_nn as nn
    wide = variant == "wide"
    if variant in ("l128", "wide"):
        dispatch("no_p")
    if variant in ("p64", "p256"):
        dispatch("p_bn=" + variant[1:])
    if wide:
        dispatch("w256_min_k=0")
    B, H, Cin, Cout = 16, 128, 64, 256
    g = torch.Generator(device="cuda").manual_seed(12)
    x = rnd((B, H, H, Cin), 1.0, g)
    w = rnd((1, 1, Cin, Cout), Cin ** -0.5, g).to(F64)
    bias = torch.randn(Cout, generator=g, device="cuda")
    wf, _ = packs(w)
    d = nn.make_desc(nn.FWD, B, Cin, 1, 1, 1, 0, 0, Cout, Cout, Cout, [nn.seg(H, H, H, H, wf, bias)])
    out = torch.empty((B, H, H, Cout), dtype=BF, device="cuda")
    stats = nn.bn_acc(B, Cout, "cuda")
    nn.conv_igemm(d, x, out, stats)
    code, name = last_kernel()
    print("kernel:", name)
    assert code in ((5, 6, 7) if wide else ((4,) if variant == "l128" else (16,))), name
    ref = conv_ref(x.to(F64), w, pt=0, pl=0) + bias.to(F64)
    torch.testing.assert_close(out.to(F64), ref, rtol=1e-2, atol=1e-2)
    o = out.to(F64)
    exp = torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1)
    torch.testing.assert_close(nn.bn_acc_value(stats), exp, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,NP", [(720, 768), (36, 64)])
def test_retina_cls_head_f32_epilogue_configs4(N, NP):
    """RetinaNet grouped class head at bs 8 / 640, C = 80 (9 anchors x 80 = 720 channels, Npad 768),
    and the box head (9 x 4 = 36 channels, Npad 64: an fp32 destination with n_store % 8 != 0):
    fp32 destination [B, P, Npad] with bias, per-level weights, 5 segments; then its data gradient
    (K = 9 x Npad) back into the packed level-major tower buffer."""
    from cvlite import ops_nn as nn
    B, S, C = 8, 640, 256
    shapes, off, P = fpn_layout(B, S)
    g = torch.Generator(device="cuda").manual_seed(13)
    act = rnd((B * P, C), 0.5, g)
    ws = [rnd((3, 3, C, N), 0.02, g).to(F64) for _ in shapes]
    bs = [torch.randn(N, generator=g, device="cuda") for _ in shapes]
    pk = [packs(w, npad=NP) for w in ws]
    segs = [nn.seg(h, w, h, w, pk[l][0], bs[l], src_base=B * off[l], src_img=h * w, dst_base=off[l], dst_img=P)
            for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, NP, N, NP, segs, dst_f32=True)
    out = torch.full((B, P, NP), 7.0, dtype=torch.float32, device="cuda")
    nn.conv_igemm(d, act, out)
    code, name = last_kernel()
    print("head kernel:", name)
    assert code in (3, 4, 5, 6, 7), name   # an LDS-DMA large tile (fp32-destination epilogue)
    a64 = act.to(F64)
    for l, (h, w) in enumerate(shapes):
        x = a64[B * off[l]:B * (off[l] + h * w)].view(B, h, w, C)
        ref = conv_ref(x, ws[l]) + bs[l].to(F64)
        got = out[:, off[l]:off[l] + h * w, :N].reshape(B, h, w, N).to(F64)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4, msg=lambda m: "level %d: %s" % (l, m))
    assert torch.all(out[..., N:] == 7.0), "columns past n_store must not be written"
    # data gradient of the head: dout [B, P, 768] bf16 (padding channels zero) -> [B*P, 256]
    dout = torch.zeros((B, P, NP), dtype=BF, device="cuda")
    dout[..., :N] = rnd((B, P, N), 1.0, g)
    dsegs = [nn.seg(h, w, h, w, pk[l][1], None, src_base=off[l], src_img=P, dst_base=B * off[l], dst_img=h * w)
             for l, (h, w) in enumerate(shapes)]
    dd = nn.make_desc(nn.DGRAD, B, NP, 3, 3, 1, 1, 1, C, C, C, dsegs)
    dx = torch.empty((B * P, C), dtype=BF, device="cuda")
    nn.conv_igemm(dd, dout, dx)
    print("head dgrad kernel:", last_kernel()[1])
    d64 = dout.to(F64)
    for l, (h, w) in enumerate(shapes):
        ref = dgrad_ref(d64[:, off[l]:off[l] + h * w, :N].reshape(B, h, w, N), ws[l])
        got = dx[B * off[l]:B * (off[l] + h * w)].view(B, h, w, C).to(F64)
        torch.testing.assert_close(got, ref, rtol=1e-2, atol=2e-2, msg=lambda m: "dgrad level %d: %s" % (l, m))


@pytest.mark.parametrize("N,LD", [(20, 32), (5, 8)], ids=["cls20", "reg5"])
def test_fcos_heads_forward_h32_configs1(N, LD, dispatch):
    """FCOS cls / reg head forward (fcos.py:85-88, 99-101: 3x3 256 -> 20 / 5, per-level weights and
    bias, five segments) at bs 16 / 512 into the image-major fp32 head output [B, P, LD], on the
    halo kernel's 256 x 32 tile (round 6; was the 128-row generic kernel); the same launch with the
    32-wide form off (CVL_DISPATCH=no_h32) must agree to fp32 accumulation-order noise."""
    from cvlite import ops_nn as nn
    B, S, C = 16, 512, 256
    shapes, off, P = fpn_layout(B, S)
    g = torch.Generator(device="cuda").manual_seed(17)
    act = rnd((B * P, C), 0.5, g)
    ws = [rnd((3, 3, C, N), 0.02, g).to(F64) for _ in shapes]
    bs = [torch.randn(N, generator=g, device="cuda") for _ in shapes]
    pk = [packs(w) for w in ws]
    segs = [nn.seg(h, w, h, w, pk[l][0], bs[l], src_base=B * off[l], src_img=h * w, dst_base=off[l], dst_img=P)
            for l, (h, w) in enumerate(shapes)]
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, 32, N, LD, segs, dst_f32=True)
    out = torch.full((B, P, LD), 7.0, dtype=torch.float32, device="cuda")
    nn.conv_igemm(d, act, out)
    code, name = last_kernel()
    print("head kernel:", name)
    assert code == 14, name                 # H64 (its 256 x 32 form)
    a64 = act.to(F64)
    for l, (h, w) in enumerate(shapes):
        x = a64[B * off[l]:B * (off[l] + h * w)].view(B, h, w, C)
        ref = conv_ref(x, ws[l]) + bs[l].to(F64)
        got = out[:, off[l]:off[l] + h * w, :N].reshape(B, h, w, N).to(F64)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4, msg=lambda m: "level %d: %s" % (l, m))
    assert torch.all(out[..., N:] == 7.0), "columns past n_store must not be written"
    dispatch("no_h32")
    out2 = torch.full((B, P, LD), 7.0, dtype=torch.float32, device="cuda")
    nn.conv_igemm(d, act, out2)
    assert last_kernel()[0] != 14
    torch.testing.assert_close(out2, out, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode,B,H,W,C,N", [("fwd", 2, 64, 64, 256, 256), ("dgrad", 3, 32, 32, 512, 256),
                                           ("fwd", 3, 8, 8, 256, 256), ("dgrad", 5, 4, 4, 256, 512),
                                           ("fwd", 2, 16, 16, 256, 256), ("fwd", 1, 64, 64, 64, 256)])
def test_x32_tile_geometries(dispatch, mode, B, H, W, C, N):
    """The 256x256 ring kernel (X32) on 3x3 tile geometries: R image rows of one image (W = 64 / 32 /
    16), several whole images per tile (8x8: 4, 4x4: 16 per tile, batches that leave the last
    tile's images partly absent), Cin 64 / 256 / 512, fwd with bias + ReLU + BN statistics and
    dgrad, against fp64."""
    from cvlite import ops_nn as nn
    dispatch("l_min_tiles=1", "l256_min_tiles=1", "no_h")
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + H + C)
    x = rnd((B, H, W, C), 1.0, g)
    if mode == "fwd":
        w = rnd((3, 3, C, N), (9 * C) ** -0.5, g).to(F64)
        wf, _ = packs(w)
        bias = torch.randn(N, generator=g, device="cuda")
        d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, W, H, W, wf, bias)], relu_out=True)
        ref = torch.relu(conv_ref(x.to(F64), w) + bias.to(F64))
    else:
        w = rnd((3, 3, N, C), (9 * C) ** -0.5, g).to(F64)      # forward conv N -> C; dgrad C -> N
        _, wd = packs(w)
        d = nn.make_desc(nn.DGRAD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, W, H, W, wd, None)])
        ref = dgrad_ref(x.to(F64), w)
    out = torch.empty((B, H, W, N), dtype=BF, device="cuda")
    stats = nn.bn_acc(B, N, "cuda") if mode == "fwd" else None
    nn.conv_igemm(d, x, out, stats)
    code, name = last_kernel()
    assert code == 7, name
    torch.testing.assert_close(out.to(F64), ref, rtol=1e-2, atol=2e-2)
    if stats is not None:
        o = out.to(F64)
        torch.testing.assert_close(nn.bn_acc_value(stats), torch.stack([o.sum((1, 2)), (o * o).sum((1, 2))], -1), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("mode,B,H,W,C,N", [("fwd", 2, 64, 64, 256, 256), ("dgrad", 3, 32, 32, 512, 256),
                                           ("fwd", 3, 8, 8, 256, 256), ("dgrad", 5, 4, 4, 256, 512),
                                           ("fwd", 2, 16, 16, 256, 512)])
def test_x32_register_epilogue_matches_c_image(dispatch, mode, B, H, W, C, N):
    """X32's SW epilogue (swapped MFMA operands, 16-B stores straight from the registers; taken by
    launches without BN statistics into bf16, the towers) against the LDS C-image epilogue
    (CVL_DISPATCH=x_no_sw) on the same tile geometries incl. mosaic tiles of whole 8x8 / 4x4 images
    and partly absent last tiles: bit-identical outputs, and both within bf16 rounding of fp64."""
    from cvlite import ops_nn as nn
    dispatch("l_min_tiles=1", "l256_min_tiles=1", "no_h")
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + H + C + 7)
    x = rnd((B, H, W, C), 1.0, g)
    if mode == "fwd":
        w = rnd((3, 3, C, N), (9 * C) ** -0.5, g).to(F64)
        wf, _ = packs(w)
        bias = torch.randn(N, generator=g, device="cuda")
        d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, W, H, W, wf, bias)], relu_out=True)
        ref = torch.relu(conv_ref(x.to(F64), w) + bias.to(F64))
    else:
        w = rnd((3, 3, N, C), (9 * C) ** -0.5, g).to(F64)
        _, wd = packs(w)
        d = nn.make_desc(nn.DGRAD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, W, H, W, wd, None)])
        ref = dgrad_ref(x.to(F64), w)
    outs = []
    for off in ("1", "0"):
        dispatch("x_no_sw=" + off)
        out = torch.full((B, H, W, N), 7.0, dtype=BF, device="cuda")
        nn.conv_igemm(d, x, out)
        code, name = last_kernel()
        assert code == 7, name
        outs.append(out)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    torch.testing.assert_close(outs[1].to(F64), ref, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("mode,B,H,C,N,stats", [("fwd", 4, 64, 128, 128, True), ("dgrad", 4, 64, 128, 128, False),
                                                ("fwd", 6, 8, 128, 128, False), ("fwd", 2, 32, 64, 128, True)])
def test_l_register_epilogue_matches_c_image(dispatch, mode, B, H, C, N, stats):
    """The L kernel's SW epilogue (128-wide tiles: swapped MFMA operands, 16-B stores from registers,
    per-tile BN statistics by DPP + one LDS combine) against its LDS C-image epilogue
    (CVL_DISPATCH=l_no_sw): the 3x3 128 -> 128 geometry of ResNet conv3_x (fwd with BN statistics,
    dgrad), whole 8x8 images per tile (no statistics) and Cin 64; outputs bit-identical, the
    statistics within fp32 summation order."""
    from cvlite import ops_nn as nn
    dispatch("no_h", "no_256", "l_min_tiles=1")
    g = torch.Generator(device="cuda").manual_seed(B * 100 + H + C + N)
    x = rnd((B, H, H, C), 1.0, g)
    if mode == "fwd":
        w = rnd((3, 3, C, N), (9 * C) ** -0.5, g).to(F64)
        wf, _ = packs(w)
        bias = torch.randn(N, generator=g, device="cuda")
        d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, H, H, H, wf, bias)], relu_out=True)
        ref = torch.relu(conv_ref(x.to(F64), w) + bias.to(F64))
    else:
        w = rnd((3, 3, N, C), (9 * C) ** -0.5, g).to(F64)
        _, wd = packs(w)
        d = nn.make_desc(nn.DGRAD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, H, H, H, wd, None)])
        ref = dgrad_ref(x.to(F64), w)
    res = []
    for off in ("1", "0"):
        dispatch("l_no_sw=" + off)
        out = torch.full((B, H, H, N), 3.0, dtype=BF, device="cuda")
        st = nn.bn_acc(B, N, "cuda") if stats else None
        nn.conv_igemm(d, x, out, st)
        code, name = last_kernel()
        assert "L" in name or "conv_igemm_l" in name, name
        torch.cuda.synchronize()
        res.append((out, nn.bn_acc_value(st) if stats else None))
    assert torch.equal(res[0][0].view(torch.int16), res[1][0].view(torch.int16))
    torch.testing.assert_close(res[1][0].to(F64), ref, rtol=1e-2, atol=2e-2)
    if stats:
        torch.testing.assert_close(res[0][1], res[1][1], rtol=2e-5, atol=1e-3)


def test_probe_arm_times_one_tower_launch(dispatch):
    """cvl_probe_arm (bench.py's in-step roofline timing): the armed X32 launch times itself from
    inside (slot[2] = 1 launch, slot[1] > 0 ticks, the workgroup counter slot[3] back at 0, the
    output bit-identical to an unarmed launch); the arm is consumed by the next conv_igemm call, so
    a launch on another kernel leaves the slot untouched and the X32 launch after it is not timed."""
    from cvlite import ops_nn as nn
    dispatch("l_min_tiles=1", "l256_min_tiles=1", "no_h")
    B, H, C, N = 2, 64, 256, 256
    g = torch.Generator(device="cuda").manual_seed(77)
    x = rnd((B, H, H, C), 1.0, g)
    w = rnd((3, 3, C, N), (9 * C) ** -0.5, g).to(F64)
    wf, _ = packs(w)
    d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, N, N, N, [nn.seg(H, H, H, H, wf, None)])
    slot = torch.zeros(4, dtype=torch.int64, device="cuda")
    ref = torch.empty((B, H, H, N), dtype=BF, device="cuda")
    nn.conv_igemm(d, x, ref)
    out = torch.empty_like(ref)
    for _ in range(3):
        nn.probe_arm(slot)
        nn.conv_igemm(d, x, out)
        assert last_kernel()[0] == 7
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    s = slot.cpu().tolist()
    assert s[2] == 3 and s[1] > 0 and s[3] == 0, s
    sec, n = nn.probe_seconds(slot)
    assert n == 3 and 0 < sec < 0.05
    # a 1x1 launch (not X32) consumes the arm and leaves the slot as it was
    w1 = rnd((1, 1, C, N), C ** -0.5, g).to(F64)
    wf1, _ = packs(w1)
    d1 = nn.make_desc(nn.FWD, B, C, 1, 1, 1, 0, 0, N, N, N, [nn.seg(H, H, H, H, wf1, None)])
    nn.probe_arm(slot)
    nn.conv_igemm(d1, x, out)
    assert last_kernel()[0] != 7
    nn.conv_igemm(d, x, out)
    torch.cuda.synchronize()
    assert slot.cpu().tolist() == s
