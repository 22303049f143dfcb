"""BN accumulators on the GPU (include/cvlite.h "BN accumulators", csrc/bn_acc.h).  Exact mode
(cvl_bn_set_exact(1)): the fused statistics of a conv launch are bit-identical across repeated
launches (integer bins: the order the atomics land in cannot matter), equal the float64 sums of the
stored outputs, and cvl_bn_acc_decode equals the host restatement of the decode bit for bit.  Default
mode (one float64 per statistic): the same sums within fp64 rounding."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _decode_host(acc):
    a = acc.cpu()
    t = torch.zeros(a.shape[:-1], dtype=torch.float64)
    for k in range(7):
        t = t + a[..., k].double() * math.ldexp(1.0, 27 + 22 * k - 150)
    return torch.where(a[..., 7] != 0, torch.full_like(t, float("nan")), t)


@pytest.fixture
def exact_mode():
    from cvlite import ops_nn as nn
    nn.set_bn_exact(True)
    assert nn.acc_slots() == nn.ACC_SLOTS
    yield
    nn.set_bn_exact(False)


@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("H,Cin,Cout,k", [(128, 64, 64, 3), (32, 256, 1024, 1), (40, 256, 256, 3)])
def test_conv_stats_across_launches(H, Cin, Cout, k, exact):
    from cvlite import ops_nn as nn
    nn.set_bn_exact(exact)
    try:
        _conv_stats(H, Cin, Cout, k, exact)
    finally:
        nn.set_bn_exact(False)


def _conv_stats(H, Cin, Cout, k, exact):
    from cvlite import ops_nn as nn
    from cvlite.layers import Conv, ParamStore
    B = 8
    st = ParamStore()
    conv = Conv(st, "c", k, Cin, Cout)
    st.finalize(torch.device("cuda", 0), seed=4)
    conv.pack()
    g = torch.Generator(device="cpu").manual_seed(11)
    x = (torch.randn((B, H, H, Cin), generator=g) * 2.0 - 0.3).to(BF).cuda()
    accs = []
    for _ in range(3):
        acc = nn.bn_acc(B, Cout, "cuda")
        z, _, _ = conv.fwd(x, B, H, H, stats=acc)
        accs.append(acc)
    torch.cuda.synchronize()
    assert accs[0].shape[-1] == (nn.ACC_SLOTS if exact else 1)
    if exact:
        assert torch.equal(accs[0], accs[1]) and torch.equal(accs[0], accs[2])
    o = z.double().reshape(B, H * H, Cout)
    ref = torch.stack([o.sum(1), (o * o).sum(1)], -1)
    val = nn.bn_acc_value(accs[0])
    torch.testing.assert_close(val, ref, rtol=1e-6, atol=1e-6 * float(ref.abs().max()))
    if exact:
        assert torch.equal(val.cpu(), _decode_host(accs[0]))
    else:
        assert torch.equal(val.cpu(), accs[0][..., 0].cpu().view(torch.float64))


def test_acc_decode_nonfinite_and_encode_roundtrip(exact_mode):
    from cvlite import ops_nn as nn
    vals = torch.tensor([[1.5, -2.25e-3], [3.0e15, 0.0], [float("inf"), 7.0]], dtype=torch.float64)
    acc = nn.bn_acc_encode(vals).cuda()
    out = nn.bn_acc_value(acc).cpu()
    assert out[0, 0] == 1.5 and out[0, 1] == -2.25e-3 and out[1, 0] == 3.0e15 and out[1, 1] == 0.0
    assert math.isnan(out[2, 0]) and out[2, 1] == 7.0
    assert torch.equal(torch.nan_to_num(out), torch.nan_to_num(_decode_host(acc)))
