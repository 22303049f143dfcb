"""The torch custom-op layer (cvlite.torch_ops): torch.ops.cvlite.* run the HIP
kernels and carry autograd, so the reference's GradientTape step (FCOS/train_fcos.py:152-174:
`model(image, training=True)` -> `model_loss` -> `grad_tape.gradient(all_losses, model_params)`)
can be written with torch.autograd.grad on the MI355X model.

* whole FCOS model: torch.autograd.grad(cls + reg + cen, model.trainable_variables) equals
  FCOSTrainer's gradient buffer for the same image bit-for-bit (same kernels);
* conv2d_nhwc forward / dx / dw / db vs float64 torch (bf16 tolerances as tests/test_gpu_conv.py);
* fcos_loss with distinct upstream gradients per image and per term vs float64 autograd of the
  oracle restatement (oracle/fcos_torch.py) (1e-4 relative, fp32 kernel);
* sgd_clip_ in place vs the restated Keras SGD + clip_by_global_norm."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_model_autograd_matches_trainer_gradient():
    from cvlite import fcos
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, S = 20, 256
    imgs, boxes, nbox = synthetic_batch(1, S, S, C, seed=31)
    gt = boxes[0, :int(nbox[0])].cpu().numpy()
    model = fcos.build_model(C)                      # seed 0
    y_true, _ = fcos.format_data(gt, np.array([S, S], np.float32), C)
    out = model(imgs, training=True)
    assert all(o.requires_grad for o in out)
    lc, lr, le = fcos.model_loss(y_true, out, (8, 16, 32, 64, 128))
    total = lc + lr + le
    grads = torch.autograd.grad(total, model.trainable_variables)
    net = FCOSNet(C, device=torch.device("cuda"), seed=0)
    tr = FCOSTrainer(net, 1, (S, S), use_graph=False)
    tr.load_batch(imgs, boxes, nbox)
    tr._fwd_bwd()
    torch.cuda.synchronize()
    np.testing.assert_allclose(tr.losses[0].cpu().numpy(), torch.stack([lc, lr, le]).detach().cpu().numpy(),
                               rtol=0, atol=0)
    st = net.store
    for name, g in zip(st.offsets, grads):
        assert torch.equal(g, st.g(name)), name
    # and the outputs of a no-grad call are plain tensors
    with torch.no_grad():
        assert not model(imgs, training=True)[0].requires_grad


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 3, 1, "same"), (2, 17, 13, 32, 40, 3, 2, "same"),
                                  (1, 12, 12, 128, 256, 1, 1, "valid")])
def test_conv2d_nhwc_op_autograd(case):
    from cvlite import torch_ops  # noqa: F401
    B, H, W, Cin, Cout, k, s, pad = case
    g = torch.Generator().manual_seed(H + Cin)
    x = (torch.randn(B, H, W, Cin, generator=g)).to(torch.bfloat16).double()
    w = (torch.randn(k, k, Cin, Cout, generator=g) * (k * k * Cin) ** -0.5).to(torch.bfloat16).double()
    b = torch.randn(Cout, generator=g).double()
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    if pad == "same":
        out_h = -(-H // s)
        th = max((out_h - 1) * s + k - H, 0)
        out_w = -(-W // s)
        tw = max((out_w - 1) * s + k - W, 0)
        xp = F.pad(xr.permute(0, 3, 1, 2), (tw // 2, tw - tw // 2, th // 2, th - th // 2))
    else:
        xp = xr.permute(0, 3, 1, 2)
    ref = F.conv2d(xp, wr.permute(3, 2, 0, 1), br, s).permute(0, 2, 3, 1)
    gy = torch.randn(ref.shape, generator=g).to(torch.bfloat16).double()
    ref.backward(gy)
    xg = x.to(torch.bfloat16).cuda().requires_grad_()
    wg = w.float().cuda().requires_grad_()
    bg = b.float().cuda().requires_grad_()
    y = torch.ops.cvlite.conv2d_nhwc(xg, wg, bg, s, pad)
    torch.testing.assert_close(y.double().cpu(), ref.detach(), rtol=1e-2, atol=1e-2)
    y.backward(gy.to(torch.bfloat16).cuda())
    torch.testing.assert_close(xg.grad.double().cpu(), xr.grad, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(wg.grad.double().cpu(), wr.grad, rtol=1e-4, atol=1e-5 * float(wr.grad.abs().max()))
    torch.testing.assert_close(bg.grad.double().cpu(), br.grad, rtol=1e-4, atol=1e-3)


def test_fcos_loss_op_autograd_per_term_weights():
    from cvlite import ops_targets as ot
    from cvlite import torch_ops  # noqa: F401
    from oracle import fcos_torch
    from cvlite.train_fcos import synthetic_batch
    C, B, S = 20, 3, 256
    _, boxes, nbox = synthetic_batch(B, S, S, C, seed=8)
    tg, _ = torch.ops.cvlite.fcos_assign(boxes, nbox, torch.full((B, 2), float(S), device="cuda"), S, S, C)
    P = tg.shape[1]
    g = torch.Generator().manual_seed(3)
    reg = torch.zeros(B, P, 8)
    reg[..., :5] = torch.randn(B, P, 5, generator=g)
    cls = torch.zeros(B, P, 32)
    cls[..., :C] = torch.randn(B, P, C, generator=g) - 2
    rg, cg = reg.cuda().requires_grad_(), cls.cuda().requires_grad_()
    losses = torch.ops.cvlite.fcos_loss(rg, cg, tg, C, 0)
    wts = torch.tensor([[2.0, 0.5, 3.0], [1.0, -1.0, 0.25], [0.0, 1.5, 1.0]])
    (losses * wts.cuda()).sum().backward()
    rr, cc = reg.double().requires_grad_(), cls.double().requires_grad_()
    tot, exp = 0.0, []
    for b in range(B):
        l = fcos_torch.packed_loss(rr[b], cc[b], tg[b].double().cpu(), C)
        exp.append([float(v) for v in l])
        tot = tot + sum(float(wts[b, i]) * l[i] for i in range(3))
    tot.backward()
    np.testing.assert_allclose(losses.detach().cpu().numpy(), np.array(exp), rtol=2e-5)
    torch.testing.assert_close(rg.grad.double().cpu(), rr.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(cg.grad.double().cpu(), cc.grad, rtol=1e-4, atol=1e-6)
    assert not rg.grad[..., 5:].any() and not cg.grad[..., C:].any()
    # the low-level wrapper agrees with the op
    l2, _, _ = ot.fcos_loss(reg.cuda(), cls.cuda(), tg, C, with_grad=False)
    torch.testing.assert_close(l2, losses.detach(), rtol=0, atol=0)


def test_sgd_clip_op():
    from cvlite import torch_ops  # noqa: F401
    g0 = torch.Generator().manual_seed(1)
    w = torch.randn(10000, generator=g0)
    gr = torch.randn(10000, generator=g0) * 3
    v = torch.randn(10000, generator=g0) * 0.1
    lr = torch.tensor([0.01])
    wd, vd = w.cuda(), v.cuda()
    torch.ops.cvlite.sgd_clip_(wd, gr.cuda(), vd, lr.cuda(), 0.9, 0.25, 1.0)
    gs = gr.double() * 0.25
    gs = gs * (1.0 / max(float(gs.norm()), 1.0))
    v_exp = 0.9 * v.double() - 0.01 * gs
    torch.testing.assert_close(vd.double().cpu(), v_exp, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(wd.double().cpu(), w.double() + v_exp, rtol=1e-5, atol=1e-6)
