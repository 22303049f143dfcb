"""CPU checks of the float64 restatements the teacher-forced launch-parity harness
(tests/launch_parity.py) compares the GPU against: the explicit im2col conv forward / data
gradient / weight gradient (TF 'same' asymmetric pads, stride 2, cropped borders) against torch's
own float64 conv + autograd, and the pool / up-sample references against torch's ops."""
import torch
import torch.nn.functional as F

import launch_parity as lp


def _same(n, k, s):
    out = -(-n // s)
    return out, max((out - 1) * s + k - n, 0) // 2


def _torch_conv(x, w, s, pt, pl, Ho, Wo):
    """NHWC / OHWI float64 conv via F.conv2d with explicit asymmetric padding."""
    xn = x.permute(0, 3, 1, 2)
    KH, KW = w.shape[1], w.shape[2]
    H, W = xn.shape[2], xn.shape[3]
    pb = max(0, (Ho - 1) * s + KH - H - pt)
    pr = max(0, (Wo - 1) * s + KW - W - pl)
    y = F.conv2d(F.pad(xn, (pl, pr, pt, pb)), w.permute(0, 3, 1, 2), stride=s)
    return y[:, :, :Ho, :Wo].permute(0, 2, 3, 1)


def test_conv_restatement_vs_torch():
    g = torch.Generator().manual_seed(0)
    for (H, W, k, s, Ci, O) in [(9, 7, 3, 1, 5, 6), (10, 11, 3, 2, 4, 3), (8, 8, 1, 2, 6, 5), (13, 13, 7, 2, 3, 4),
                                (4, 4, 3, 2, 2, 2)]:
        (Ho, pt), (Wo, pl) = _same(H, k, s), _same(W, k, s)
        x = torch.randn((2, H, W, Ci), generator=g, dtype=torch.float64, requires_grad=True)
        w = torch.randn((O, k, k, Ci), generator=g, dtype=torch.float64, requires_grad=True)
        y = _torch_conv(x, w, s, pt, pl, Ho, Wo)
        torch.testing.assert_close(lp.conv_fwd64(x.detach(), w.detach(), s, pt, pl, Ho, Wo), y.detach())
        dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
        gx, gw = torch.autograd.grad(y, (x, w), dy)
        torch.testing.assert_close(lp.conv_dgrad64(dy, w.detach(), s, pt, pl, H, W), gx)
        torch.testing.assert_close(lp.conv_wgrad64(x.detach(), dy, k, k, s, pt, pl), gw.permute(1, 2, 3, 0))


def test_pool_and_upsample_restatements():
    g = torch.Generator().manual_seed(1)
    a = torch.randn((2, 9, 8, 3), generator=g).clamp_min(0).to(torch.bfloat16)
    y, arg = lp._pool3_ref(a)
    ref = F.max_pool2d(F.pad(a.float().permute(0, 3, 1, 2), (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, ref)
    # argmax is the first maximum in window order; the backward routes dy there
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx = lp._pool3_bwd_ref(dy, arg, 9, 8)
    ap = F.pad(a.double().permute(0, 3, 1, 2), (1, 1, 1, 1)).requires_grad_()
    win = F.unfold(ap, 3, stride=2)
    # reference gradient: route to the first max tap, then drop the padding rows / cols
    B, C = 2, 3
    w9 = win.view(B, C, 9, -1)
    first = (w9 == w9.max(2, keepdim=True).values).double()
    first = first * (first.cumsum(2) == 1).double()
    gcols = (first * dy.permute(0, 3, 1, 2).reshape(B, C, 1, -1)).view(B, C * 9, -1)
    gpad = F.fold(gcols, (ap.shape[2], ap.shape[3]), 3, stride=2)
    torch.testing.assert_close(dx, gpad[:, :, 1:-1, 1:-1].permute(0, 2, 3, 1))
    # bilinear x2 (Keras half-pixel): out[2i] = .75 x[i] + .25 x[i-1], out[2i+1] = .75 x[i] + .25 x[i+1]
    # (edges clamped)
    p = torch.randn((1, 1, 4, 1), generator=g, dtype=torch.float64)
    up = lp._bilinear_up2(p)[0, 0, :, 0]
    x = p[0, 0, :, 0]
    xm, xp = torch.cat([x[:1], x[:-1]]), torch.cat([x[1:], x[-1:]])
    ref = torch.stack([0.75 * x + 0.25 * xm, 0.75 * x + 0.25 * xp], 1).reshape(-1)
    torch.testing.assert_close(up, ref)


def test_bn_affine_mask_is_fma_exact():
    g = torch.Generator().manual_seed(2)
    z = torch.randn(4096, generator=g).to(torch.bfloat16)
    m, rs, ga, be = torch.tensor(0.1), torch.tensor(1.7), torch.tensor(0.9), torch.tensor(-0.05)
    a, xh = lp.bn_affine32(z, m, rs, ga, be)
    exact = ga.double() * ((z.float() - m) * rs).double() + be.double()
    assert torch.equal(a > 0, exact > 0)
