"""BN -> ReLU folded into a 1x1 consumer (include/cvlite.h cvl_conv_igemm_fold / cvl_conv_wgrad_fold;
Keras ResNet block1's conv2 BN + ReLU feeding conv3, behind FCOS/fcos.py:30-35): the fused forward
(finalize inside the launch + the BN applied to the A operand in registers) is bit-identical to
cvl_bn_finalize_apply + cvl_conv_igemm on the stored input -- output, (mean, rstd), running
statistics -- its conv BN statistics agree to float64 rounding, and the fused weight gradient is
bit-identical to cvl_conv_wgrad on the stored input.  Shapes: the bottleneck conv3 launches of
the 512x512 step (K = filters, N = 4 * filters) at reduced batch, and one that must decline
(H*W % 256 != 0: CVL_ENOTTAKEN, nothing written)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _unit(cin, cout, seed):
    from cvlite.layers import BatchNorm, Conv, ParamStore
    st = ParamStore()
    conv = Conv(st, "c3", 1, cin, cout)
    bn = BatchNorm(st, "bn2", cin)
    st.finalize(torch.device("cuda", 0), seed=seed)
    g = torch.Generator().manual_seed(seed)
    st.p(bn.gname).copy_((torch.rand(cin, generator=g) + 0.5).cuda())
    st.p(bn.bname).copy_((torch.randn(cin, generator=g) * 0.5).cuda())
    bn.init_buffers(torch.device("cuda", 0)) if hasattr(bn, "init_buffers") else None
    conv.pack()
    return st, conv, bn


@pytest.mark.parametrize("B,H,cin", [(4, 64, 64), (4, 32, 128), (8, 16, 256), (16, 16, 512)])
def test_fold_forward_and_wgrad_bit_identical(B, H, cin):
    from cvlite import ops_nn as nn
    from cvlite.layers import FoldedInput
    cout = 4 * cin
    st, conv, bn = _unit(cin, cout, seed=cin + H)
    g = torch.Generator().manual_seed(7 * cin + B)
    z = (torch.randn((B, H, H, cin), generator=g) * 1.5 + 0.3).to(BF).cuda()
    zd = z.double().reshape(B, H * H, cin)
    stats = nn.bn_acc_encode(torch.stack([zd.sum(1), (zd * zd).sum(1)], -1)).cuda()
    dy = (torch.randn((B, H, H, cout), generator=g) * 0.05).to(BF).cuda()
    res = []
    for fused in (False, True):
        rm, rv = torch.full((cin,), 0.2, device="cuda"), torch.full((cin,), 0.7, device="cuda")
        bn.run_mean, bn.run_var = rm, rv
        mr = torch.empty((B, cin, 2), device="cuda")
        f = FoldedInput(z, stats.clone(), mr, bn)
        cst = nn.bn_acc(B, cout, "cuda")
        if fused:
            out, x = conv.fwd_folded(f, B, H, H, stats=cst)
            assert x is f, "the fused forward declined a qualifying launch"
        else:
            x = f.finalize_apply(B, H * H)
            out, _, _ = conv.fwd(x, B, H, H, stats=cst)
        dw = torch.empty_like(conv.dw)
        with nn.deferred_wgrad():
            conv.wgrad(x, dy, B, H, H, dw=dw, bias=False)
            nn.wgrad_flush()
        torch.cuda.synchronize()
        res.append((out.view(torch.int16), mr, rm, rv, dw, nn.bn_acc_value(cst)))
    (o0, m0, rm0, rv0, w0, s0), (o1, m1, rm1, rv1, w1, s1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(m0, m1) and torch.equal(rm0, rm1) and torch.equal(rv0, rv1)
    assert torch.equal(w0, w1)
    torch.testing.assert_close(s1, s0, rtol=1e-12, atol=1e-9 * float(s0.abs().max()))


def test_fold_declines_when_tiles_straddle_images():
    from cvlite import ops_nn as nn
    from cvlite.layers import FoldedInput
    B, H, cin = 2, 20, 64                    # H*W = 400: a 256-row tile would span two images
    st, conv, bn = _unit(cin, 256, seed=3)
    z = torch.randn((B, H, H, cin)).to(BF).cuda()
    zd = z.double().reshape(B, H * H, cin)
    stats = nn.bn_acc_encode(torch.stack([zd.sum(1), (zd * zd).sum(1)], -1)).cuda()
    mr = torch.full((B, cin, 2), 7.0, device="cuda")
    f = FoldedInput(z, stats, mr, bn)
    out, x = conv.fwd_folded(f, B, H, H, stats=nn.bn_acc(B, 256, "cuda"))
    assert x is not f                        # the unfused form ran: the input was materialised
    ref, _, _ = conv.fwd(x, B, H, H)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
