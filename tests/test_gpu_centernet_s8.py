"""CenterNet ResNet stride-8 multi-scale (CenterNet/tf_centernet_resnet_s8.py +
train_centernet_crowdhuman.py) on the GPU.

  * targets: cvl_centernet_s8_assign bit-exact vs the reference's format_data outputs
    (tests/golden/golden_centernet_s8.npz) and vs the oracle on a larger batch;
  * loss: cvl_centernet_s8_loss vs the reference's model_loss (rtol 2e-5), gradient vs float64
    autograd;
  * corners: prediction_to_corners (fp32 TF math) exact vs its restatement;
  * whole graph (ResNet-101, 128x128, B = 2, residual-branch gammas damped as test_gpu_model.py so
    the random-init graph is not chaotic) vs the bf16-storage oracle; train steps through the graph.
"""
import math

import numpy as np
import pytest
import torch

from oracle import centernet_s8_ref as s8

pytestmark = pytest.mark.gpu
SCALES = [32.0, 64.0, 128.0, 256.0, 512.0]


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_s8_assign_vs_reference(golden):
    from cvlite import tf_centernet_resnet_s8 as m
    d = golden("centernet_s8")
    for i in range(12):
        raw, img = (int(v) for v in d["case_%d_dims" % i])
        out, n = m.format_data(d["case_%d_rows" % i], SCALES, [raw, raw], 3, img_pad=[img, img])
        np.testing.assert_array_equal(out, d["case_%d_out" % i])
        assert n == int(d["case_%d_n" % i])


def test_s8_assign_batched_vs_oracle():
    from cvlite import ops_targets as ot
    rng = np.random.default_rng(21)
    B, C, nmax, img = 8, 4, 100, 512
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = rng.integers(0, nmax + 1, B).astype(np.int32)
    nbox[0], nbox[1] = 0, 1
    dims = np.zeros((B, 2), np.float32)
    for b in range(B):
        n = nbox[b]
        boxes[b, :n, 0:2] = rng.uniform(-0.02, 1.02, (n, 2))
        boxes[b, :n, 2:4] = np.exp(rng.uniform(np.log(0.005), np.log(1.3), (n, 2)))   # some fit no scale
        boxes[b, :n, 4] = rng.integers(0, C, n)
        dims[b] = [448 + 8 * b, 448 + 8 * b]
    tg = ot.centernet_s8_assign(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(),
                                torch.from_numpy(dims).cuda(), (img, img), C, SCALES)
    tg = tg.cpu().numpy()
    for b in range(B):
        ref, _ = s8.format_data(boxes[b, :nbox[b]], SCALES, [float(dims[b, 0]), float(dims[b, 1])], C,
                                img_pad=[img, img])
        np.testing.assert_array_equal(tg[b], ref)


def test_s8_loss_vs_reference_and_grad(golden):
    from cvlite import ops_targets as ot
    from cvlite import tf_centernet_resnet_s8 as m
    d = golden("centernet_s8")
    yt, rl, cl = d["loss_y"], d["loss_reg_logits"], d["loss_cls_logits"]
    B, S0, S1, ns, R = yt.shape
    C = R - 4
    P = S0 * S1
    reg = torch.from_numpy(rl).reshape(B, P, ns * 4).cuda()
    cls = torch.from_numpy(cl).reshape(B, P, ns * C).cuda()
    losses, dr, dc = ot.centernet_s8_loss(reg, cls, torch.from_numpy(yt).cuda().view(B, P, ns, R), C, ns,
                                          cls_scale=1.0, reg_scale=1.0)
    np.testing.assert_allclose(losses.double().sum(0).cpu().numpy(), d["loss_out"], rtol=2e-5)
    pred = np.concatenate([1.0 / (1.0 + np.exp(-rl.astype(np.float64))), cl], -1).astype(np.float32)
    np.testing.assert_allclose(m.model_loss(yt, pred), d["loss_out"], rtol=1e-4)
    tr = torch.from_numpy(rl).double().requires_grad_()
    tc = torch.from_numpy(cl).double().requires_grad_()
    lc, lr = s8.model_loss_torch(torch.from_numpy(yt).double(), tr, tc)
    (lc + lr).backward()
    gr = dr.float().cpu()[..., :ns * 4].reshape(B, S0, S1, ns, 4).double()
    gc = dc.float().cpu()[..., :ns * C].reshape(B, S0, S1, ns, C).double()
    assert torch.allclose(gr, tr.grad, rtol=1e-2, atol=1e-6) and torch.allclose(gc, tc.grad, rtol=1e-2, atol=1e-6)
    assert not dr[..., ns * 4:].any() and not dc[..., ns * C:].any()


def test_s8_prediction_to_corners():
    from cvlite import tf_centernet_resnet_s8 as m
    rng = np.random.default_rng(3)
    xy = rng.uniform(0, 1, (6, 7, 5, 4)).astype(np.float32)
    got = m.prediction_to_corners(xy, SCALES, stride=8)
    f32 = np.float32
    gy, gx = np.meshgrid(np.arange(6, dtype=f32), np.arange(7, dtype=f32), indexing="ij")
    for s in range(5):
        yc = (gy + xy[:, :, s, 0]) * f32(8)
        xc = (gx + xy[:, :, s, 1]) * f32(8)
        bh = xy[:, :, s, 2] * f32(SCALES[s])
        bw = xy[:, :, s, 3] * f32(SCALES[s])
        np.testing.assert_array_equal(got[:, :, s, 0], yc - bh / f32(2))
        np.testing.assert_array_equal(got[:, :, s, 1], xc - bw / f32(2))
        np.testing.assert_array_equal(got[:, :, s, 2], yc + bh / f32(2))
        np.testing.assert_array_equal(got[:, :, s, 3], xc + bw / f32(2))


def _damp(net, factor):
    for k in net.store.offsets:
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(factor)


def _targets(rng, B, S, C, n=5):
    t = np.zeros((B, S, S, 5, 4 + C), np.float32)
    for b in range(B):
        for _ in range(n):
            i, j, s = int(rng.integers(0, S)), int(rng.integers(0, S)), int(rng.integers(0, 5))
            t[b, i, j, s, :4] = rng.uniform(0, 1, 4)
            t[b, i, j, s, 4 + int(rng.integers(0, C))] = 1.0
    return torch.from_numpy(t)


def test_s8_forward_loss_backward_vs_oracle():
    from cvlite import ops_targets as ot
    from cvlite.centernet_s8_net import CenterNetS8Net
    from oracle.model_ref import emulate_bf16
    C, B, D, ns = 2, 2, 128, 5
    net = CenterNetS8Net(C, n_scales=ns, seed=1)
    _damp(net, 0.25)
    net.pack()
    params = net.store.state_dict()
    x = torch.rand(B, D, D, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1
    S = D // 8
    tg = _targets(np.random.default_rng(1), B, S, C)
    reg, cls = net.forward(x.cuda())
    d_reg = torch.zeros((B, S * S, net.reg_ld), dtype=torch.bfloat16, device="cuda")
    d_cls = torch.zeros((B, S * S, net.cls_ld), dtype=torch.bfloat16, device="cuda")
    losses, _, _ = ot.centernet_s8_loss(reg, cls, tg.cuda().view(B, S * S, ns, -1), C, ns, d_reg=d_reg, d_cls=d_cls)
    net.backward(d_reg, d_cls)
    torch.cuda.synchronize()
    with emulate_bf16():
        c16, r16, g16, (or16, oc16) = s8.loss_and_grads(params, x, tg, C, ns)
    c32, r32, g32, (or32, oc32) = s8.loss_and_grads(params, x, tg, C, ns)
    gr = reg.cpu().view(B, S, S, ns, 4)
    gc = cls.cpu().view(B, S, S, ns, C)
    e_r, e_c = rel(gr, or16), rel(gc, oc16)
    print("reg %.4f cls %.4f vs bf16-oracle | bf16 vs fp32: %.4f %.4f" % (e_r, e_c, rel(or16, or32), rel(oc16, oc32)))
    assert e_r < max(2e-2, 1.5 * rel(or16, or32)) and e_c < max(2e-2, 1.5 * rel(oc16, oc32))
    lc, lr = float(losses[:, 0].sum()), float(losses[:, 1].sum())
    # losses: bounded like the outputs, by the oracle's own bf16-storage divergence on each term
    bc = max(2e-2, 1.5 * abs(c16 - c32) / abs(c32))
    br = max(2e-2, 1.5 * abs(r16 - r32) / abs(r32))
    print("loss rel: cls %.4f (bound %.4f) reg %.4f (bound %.4f)" % (abs(lc - c16) / abs(c16), bc,
                                                                       abs(lr - r16) / abs(r16), br))
    assert abs(lc - c16) / abs(c16) < bc and abs(lr - r16) / abs(r16) < br
    big = max(float(v.norm()) for v in g32.values())
    excess = []
    for k, gref in g32.items():
        if float(gref.norm()) < 1e-3 * big or k.endswith("_conv/bias"):
            continue
        e_gpu, e_emu = rel(net.store.g(k).cpu(), gref), rel(g16[k], gref)
        # head kernels see a handful of positive cells: their gradients are the noisiest tensors
        excess.append((e_gpu - (2.0 * e_emu + 0.05), e_gpu, e_emu, k))
    excess.sort(reverse=True)
    print("worst (excess, gpu, bf16-oracle, tensor):", excess[:4])
    assert excess[0][0] <= 0, excess[:4]


def test_s8_train_steps_vs_oracle():
    from cvlite.centernet_s8_net import CenterNetS8Net
    from cvlite.train_centernet_s8 import S8Trainer
    from oracle.model_ref import emulate_bf16
    C, B, D, ns = 1, 2, 128, 5
    net = CenterNetS8Net(C, n_scales=ns, seed=2)
    _damp(net, 0.25)
    net.pack()
    p0 = net.store.state_dict()
    tr = S8Trainer(net, B, D, n_max=8, init_lr=0.01)
    rng = np.random.default_rng(6)
    boxes = np.zeros((B, 8, 5), np.float32)
    nbox = np.full(B, 5, np.int32)
    boxes[:, :5, 0:2] = rng.uniform(0.2, 0.8, (B, 5, 2))
    boxes[:, :5, 2:4] = np.exp(rng.uniform(np.log(0.05), np.log(0.8), (B, 5, 2)))
    imgs = torch.rand(B, D, D, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1
    P = {k: v.clone() for k, v in p0.items()}
    M = {k: torch.zeros_like(v) for k, v in P.items()}
    tg = torch.stack([torch.from_numpy(s8.format_data(boxes[b, :5], SCALES, [D, D], C, img_pad=[D, D])[0])
                      for b in range(B)])
    # the focal sum is dominated by the few largest negative logits, so it amplifies the logits'
    # bf16-level differences (the logits themselves are bounded by the forward test above; the loss
    # kernel is exact on given logits, test_s8_loss_vs_reference_and_grad): bound the loss by 4x the
    # distance bf16 storage alone puts between the oracle and itself
    c32, r32, _, _ = s8.loss_and_grads(P, imgs, tg, C, ns)
    with emulate_bf16():
        c16, r16, _, _ = s8.loss_and_grads(P, imgs, tg, C, ns)
    own_c, own_r = abs(c16 - c32) / abs(c32), abs(r16 - r32) / abs(r32)
    for it in range(2):
        tr.load_batch(imgs.cuda(), torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda())
        losses = tr.step().double().sum(0).cpu()
        assert torch.equal(tr.targets.cpu(), tg)
        with emulate_bf16():
            c, r = s8.train_step_reference(P, M, imgs, tg, C, ns, 0.01)
        print("step %d: gpu %.4f %.4f | oracle %.4f %.4f | own %.4f %.4f" % (it, losses[0] / B, losses[1] / B, c, r,
                                                                          own_c, own_r))
        # after one SGD step the trajectories are chaotic: fp32 accumulation-order differences alone
        # (2.6e-7 rel in the head outputs: the 32-wide halo head kernel vs the generic one) move the
        # second step's reg loss by 1.3 % (1.9903 vs 2.0170, oracle 1.8988; round 6 measurement)
        tol_r = 5e-2 if it == 0 else 8e-2
        assert abs(float(losses[0]) / B - c) / abs(c) < max(3e-2, 4 * own_c)
        assert abs(float(losses[1]) / B - r) / max(abs(r), 1e-6) < max(tol_r, 4 * own_r)
    assert torch.isfinite(net.store.flat).all()
    agree = tot = 0
    for k in P:
        dg = net.store.p(k).detach().cpu().double() - p0[k].double()
        dr = P[k].double() - p0[k].double()
        m = dr.abs() > 1e-7
        agree += int(((dg > 0) == (dr > 0))[m].sum())
        tot += int(m.sum())
    print("update sign agreement %.4f" % (agree / max(tot, 1)))
    assert agree / tot > 0.8
