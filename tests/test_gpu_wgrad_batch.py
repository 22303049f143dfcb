"""GPU parity of the batched weight gradient (cvl_conv_wgrad_batch, round 6): the 1x1 weight
gradients of a ResNet stage in one launch -- the per-image gradient accumulation of
FCOS/train_fcos.py:173-176 for the Keras ResNet50 1x1 convs behind FCOS/fcos.py:30-46.

Reference: dW[ci][co] = sum over rows of x[row, ci] * dy[row, co] in float64 on the same bf16
operands (strided rows for the stride-2 1x1 convs).  Tolerance (fp32 output of an fp32 sum of
bf16 products over M rows): max |got - ref| <= 2e-5 x max |ref|.  The batched form must also agree
with the one-conv calls to the same bound, be bit-identical run to run, and give the same bits with
its split reductions deferred (cvl_wgrad_defer) or not."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F64 = torch.float64

# (B, input H = W, stride, Cin, Cout[, k]): the ResNet-50 1x1 shapes at reduced batch, a 64-channel K
# (half of the 128-wide tile idle), a 64-wide output, stride-2 projections, the ResNet 3x3 unit shapes
# (batched on the halo weight-gradient kernel) and a 3x3 stride-2 problem (neither batched kernel
# takes it: it runs as its own cvl_conv_wgrad inside the call)
PROBLEMS = [(4, 32, 1, 1024, 256), (4, 32, 1, 256, 1024), (4, 64, 2, 512, 1024), (2, 128, 1, 64, 256),
            (2, 128, 1, 64, 64), (8, 16, 1, 2048, 512), (4, 64, 2, 256, 128), (2, 32, 1, 256, 256, 3),
            (4, 16, 1, 512, 512, 3), (2, 64, 1, 128, 128, 3), (2, 128, 1, 64, 64, 3), (2, 16, 2, 256, 256, 3)]


def build(seed=0):
    from cvlite import ops_nn as nn
    g = torch.Generator(device="cuda").manual_seed(seed)
    descs, xs, dys, dws, refs = [], [], [], [], []
    for p in PROBLEMS:
        B, H, st, cin, cout = p[:5]
        k = p[5] if len(p) > 5 else 1
        pad = k // 2
        Ho = (H + st - 1) // st
        x = (torch.randn((B, H, H, cin), generator=g, device="cuda") * 0.5).to(BF)
        dy = (torch.randn((B, Ho, Ho, cout), generator=g, device="cuda") * 0.5).to(BF)
        npad = (cout + 63) // 64 * 64
        wf = torch.zeros((npad, k * k * cin), dtype=BF, device="cuda")
        d = nn.make_desc(nn.FWD, B, cin, k, k, st, pad, pad, npad, cout, cout, [nn.seg(Ho, Ho, H, H, wf, None)])
        xp = torch.nn.functional.pad(x.double(), (0, 0, pad, pad, pad, pad))
        ref = torch.zeros((k, k, cin, cout), dtype=F64, device="cuda")
        for r in range(k):
            for s in range(k):
                patch = xp[:, r:r + st * (Ho - 1) + 1:st, s:s + st * (Ho - 1) + 1:st, :]
                ref[r, s] = patch.reshape(-1, cin).t() @ dy.double().reshape(-1, cout)
        descs.append(d)
        xs.append(x)
        dys.append(dy)
        dws.append(torch.full((k * k * cin * cout,), float("nan"), dtype=torch.float32, device="cuda"))
        refs.append(ref.reshape(-1))
    return descs, xs, dys, dws, refs


def close(got, ref):
    err = float((got.double() - ref).abs().max())
    return err <= 2e-5 * float(ref.abs().max()), err


@pytest.fixture(params=["", "wgb_no_h,wgb_no_256"])
def dispatch(request, monkeypatch):
    """'' the production form; the 128-wide-only / unbatched-3x3 forms"""
    monkeypatch.setenv("CVL_DISPATCH", request.param)
    return request.param


def test_wgrad_batch_matches_float64_and_single_calls(dispatch):
    from cvlite import _lib, ops_nn as nn
    descs, xs, dys, dws, refs = build()
    nn.conv_wgrad_batch(descs, xs, dys, dws)
    assert _lib.load().cvl_conv_igemm_last_kernel() in (11, 15, 9, 10, 8)
    torch.cuda.synchronize()
    for i, (dw, ref) in enumerate(zip(dws, refs)):
        ok, err = close(dw, ref)
        assert ok, "problem %d %s: max err %.3g" % (i, PROBLEMS[i], err)
    singles = [torch.empty_like(d) for d in dws]
    for d, x, dy, dw in zip(descs, xs, dys, singles):
        nn.conv_wgrad(d, x, dy, dw)
    torch.cuda.synchronize()
    for i, (a, b, ref) in enumerate(zip(dws, singles, refs)):
        err = float((a.double() - b.double()).abs().max())
        assert err <= 2e-5 * float(ref.abs().max()), "problem %d: batch vs single %.3g" % (i, err)


def test_wgrad_batch_deterministic_and_deferral_invariant(dispatch):
    from cvlite import ops_nn as nn
    descs, xs, dys, dws, refs = build(seed=3)
    nn.conv_wgrad_batch(descs, xs, dys, dws)
    first = [d.clone() for d in dws]
    for d in dws:
        d.fill_(float("nan"))
    with nn.deferred_wgrad():
        nn.conv_wgrad_batch(descs, xs, dys, dws)
        nn.wgrad_flush()
    torch.cuda.synchronize()
    for a, b in zip(first, dws):
        assert torch.equal(a, b)


def test_wgrad_batch_beta_accumulates():
    from cvlite import ops_nn as nn
    descs, xs, dys, dws, refs = build(seed=5)
    for d in dws:
        d.fill_(0.5)
    nn.conv_wgrad_batch(descs, xs, dys, dws, beta=1.0)
    torch.cuda.synchronize()
    for i, (dw, ref) in enumerate(zip(dws, refs)):
        ok, err = close(dw, ref + 0.5)
        assert ok, "problem %d: max err %.3g" % (i, err)


def test_wgrad_batch_more_than_one_launch_group(dispatch):
    """More eligible problems than one launch takes (16): several launches, same results."""
    from cvlite import ops_nn as nn
    descs, xs, dys, dws, refs = build(seed=7)
    n = len(descs)
    reps = 3
    D = descs * reps
    X = xs * reps
    Y = dys * reps
    W = [torch.empty_like(d) for _ in range(reps) for d in dws]
    nn.conv_wgrad_batch(D, X, Y, W)
    torch.cuda.synchronize()
    for j, dw in enumerate(W):
        ok, err = close(dw, refs[j % n])
        assert ok, "copy %d problem %d: max err %.3g" % (j // n, j % n, err)
