"""GPU parity of the FCOS-center target kernel (FCOS/fcos_center.py:149-317) against the
reference's own outputs (tests/golden/golden_fcos_center.npz): bit-exact maps and counts, per image
and batched; plus a full-size batched case vs the oracle restatement."""
import numpy as np
import pytest
import torch

from oracle import fcos_ref

pytestmark = pytest.mark.gpu


def test_fcos_center_assign_bit_exact_vs_reference(golden):
    from cvlite import fcos_center
    d = golden("fcos_center")
    i = 0
    while "case_%d_cfg" % i in d:
        D, co = (int(v) for v in d["case_%d_cfg" % i])
        outs, nt = fcos_center.format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                           img_pad=[D, D], center_only=bool(co))
        assert nt == list(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(outs[l], d["case_%d_L%d" % (i, l)])
        i += 1
    assert i == 24


@pytest.mark.parametrize("center_only", [True, False])
def test_fcos_center_assign_batched_vs_oracle(center_only):
    from cvlite import fcos_center
    rng = np.random.default_rng(11)
    B, D, C, nmax = 16, 512, 20, 48
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = rng.integers(0, nmax + 1, B).astype(np.int32)
    for b in range(B):
        n = nbox[b]
        hw = np.exp(rng.uniform(np.log(4 / D), np.log(0.95), (n, 2)))
        boxes[b, :n, 2:4] = hw
        boxes[b, :n, 0] = rng.uniform(hw[:, 0] / 2, 1 - hw[:, 0] / 2)
        boxes[b, :n, 1] = rng.uniform(hw[:, 1] / 2, 1 - hw[:, 1] / 2)
        boxes[b, :n, 4] = rng.integers(0, C, n)
    dims = np.full((B, 2), D, np.float32)
    tg, nt = fcos_center.format_data_batched(torch.tensor(boxes).cuda(), torch.tensor(nbox).cuda(),
                                             torch.tensor(dims).cuda(), (D, D), C, center_only=center_only)
    tg, nt = tg.cpu().numpy(), nt.cpu().numpy()
    for b in range(B):
        outs, cnt = fcos_ref.center_format_data(boxes[b, :nbox[b]], dims[b], C, img_pad=[D, D],
                                                center_only=center_only)
        assert list(nt[b]) == cnt
        np.testing.assert_array_equal(tg[b], fcos_ref.pack_targets(outs))


def test_fcos_center_train_step():
    """train_fcos_center_voc.py's step: centre targets -> the FCOS network, fused loss, SGD; the
    loss equals the fused loss of the same predictions on cvl_fcos_center_assign's targets."""
    from cvlite import ops_targets as ot
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    net = FCOSNet(20, device=torch.device("cuda", 0), seed=0)
    tr = FCOSTrainer(net, 2, (128, 128), use_graph=False, targets="center")
    imgs, boxes, nbox = synthetic_batch(2, 128, 128, 20, seed=3)
    tr.load_batch(imgs, boxes, nbox)
    tg, _ = ot.fcos_center_assign(tr.boxes, tr.nbox, tr.img_dim, (128, 128), 20, center_only=True)
    reg, cls = net.forward(tr.images)
    ref, _, _ = ot.fcos_loss(reg, cls, tg, 20, with_grad=False)
    tr.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(tr.losses, ref, rtol=1e-6, atol=0)
    assert torch.isfinite(net.store.flat).all()


# ---- fcos_center_v1 targets / decode, centre-variant loss, the centre network ---------------------
def test_fcos_center_v1_assign_and_decode_vs_reference(golden):
    """fcos_center_v1.format_data (:149-281) and prediction_to_corners (:124-147): bit-exact vs the
    reference's own outputs (tests/golden/golden_fcos_center_v1.npz)."""
    from cvlite import fcos_center_v1
    d = golden("fcos_center_v1")
    for i in range(16):
        D = int(d["case_%d_D" % i])
        outs, nt = fcos_center_v1.format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                              img_pad=[D, D])
        assert nt == list(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(outs[l], d["case_%d_L%d" % (i, l)])
    got = fcos_center_v1.prediction_to_corners(torch.from_numpy(d["p2c_in"]).cuda(), 320.0, 16)
    np.testing.assert_array_equal(got, d["p2c_out"])


def test_fcos_center_v1_assign_batched_vs_oracle():
    """Full-size batch (16 x 512^2, up to 48 boxes, unsorted areas and shared centroid cells) vs the
    oracle restatement, bit-exact; empty images included."""
    from cvlite import fcos_center_v1
    rng = np.random.default_rng(12)
    B, D, C, nmax = 16, 512, 20, 48
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = rng.integers(0, nmax + 1, B).astype(np.int32)
    nbox[3] = 0
    for b in range(B):
        n = nbox[b]
        hw = np.exp(rng.uniform(np.log(4 / D), np.log(0.95), (n, 2)))
        boxes[b, :n, 2:4] = hw
        boxes[b, :n, 0] = rng.uniform(hw[:, 0] / 2, 1 - hw[:, 0] / 2)
        boxes[b, :n, 1] = rng.uniform(hw[:, 1] / 2, 1 - hw[:, 1] / 2)
        boxes[b, :n, 4] = rng.integers(0, C, n)
    dims = np.full((B, 2), D, np.float32)
    tg, nt = fcos_center_v1.format_data_batched(torch.tensor(boxes).cuda(), torch.tensor(nbox).cuda(),
                                                torch.tensor(dims).cuda(), (D, D), C)
    tg, nt = tg.cpu().numpy(), nt.cpu().numpy()
    for b in range(B):
        outs, cnt = fcos_ref.center_v1_format_data(boxes[b, :nbox[b]], dims[b], C, img_pad=[D, D])
        assert list(nt[b]) == cnt
        np.testing.assert_array_equal(tg[b], fcos_ref.pack_targets(outs))


def test_centre_losses_vs_reference_and_grad(golden):
    """fcos_center_v1.model_loss and fcos_center.model_loss(cen_type='focal') through the fused kernel
    vs the reference's outputs (rtol 2e-5, fp32 kernel vs the TF fp32 goldens); the training layout
    (v1: sigmoid inside the kernel, centerness logit in class column round_up(C, 8)) vs the same
    goldens, its gradients vs float64 autograd (oracle/fcos_torch.centre_packed_loss)."""
    from cvlite import fcos_center, fcos_center_v1
    from cvlite import ops_targets as ot
    from oracle import fcos_torch
    d = golden("fcos_center_v1")
    C, cc, ld = 20, 24, 64
    for i in (1, 5, 9):
        yt = [d["case_%d_L%d" % (i, l)] for l in range(5)]
        raw = [d["loss_%d_raw_L%d" % (i, l)] for l in range(5)]
        sig = []
        for r in raw:
            q = r.copy()
            q[..., :4] = torch.sigmoid(torch.from_numpy(r[..., :4])).numpy()
            sig.append(q)
        got = [float(v) for v in fcos_center_v1.model_loss(yt, sig)]
        np.testing.assert_allclose(got, d["loss_%d_out" % i], rtol=2e-5)
        got = [float(v) for v in fcos_center.model_loss(yt, raw, cen_type="focal")]
        np.testing.assert_allclose(got, d["loss_%d_center_focal" % i], rtol=2e-5)
        tgt = fcos_ref.pack_targets(yt)
        pr = np.concatenate([r[0].reshape(-1, 5 + C) for r in raw], 0)
        N = pr.shape[0]
        reg = np.zeros((N, 8), np.float32)
        reg[:, :4] = pr[:, :4]
        cls = np.zeros((N, ld), np.float32)
        cls[:, :C], cls[:, cc] = pr[:, 5:], pr[:, 4]
        losses, dreg, dcls = ot.fcos_loss(torch.from_numpy(reg)[None].cuda(), torch.from_numpy(cls)[None].cuda(),
                                          torch.from_numpy(tgt)[None].cuda(), C, grad_scale=0.5, cen_type="focal",
                                          reg_sigmoid=True, cen_in_cls=True)
        np.testing.assert_allclose(losses.cpu().numpy()[0], d["loss_%d_out" % i], rtol=2e-5)
        tr = torch.from_numpy(reg).double().requires_grad_()
        tc = torch.from_numpy(cls).double().requires_grad_()
        lc, lr, le = fcos_torch.centre_packed_loss(tr, tc[:, cc], tc, torch.from_numpy(tgt).double(), C,
                                                   cen_type="focal", reg_sigmoid=True)
        (0.5 * (lc + lr + le)).backward()
        np.testing.assert_allclose(dreg.cpu().numpy()[0], tr.grad.numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dcls.cpu().numpy()[0], tc.grad.numpy(), rtol=1e-4, atol=1e-6)
        dc = dcls.cpu().numpy()[0]
        assert not dreg[0, :, 4:].any() and not dc[:, C:cc].any() and not dc[:, cc + 1:].any()


def _bf(t):
    return t.to(torch.bfloat16).double()


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("v1", [False, True])
def test_fcos_center_net_heads_vs_torch(v1):
    """FCOSCenterNet heads (fcos_center.py:85-116): forward of the class / centerness / regression
    convs on random bf16 tower activations, and the backward (bias and weight gradients, the cls
    tower's data gradient through the combined class + centerness kernel, the reg tower's) vs float64
    torch autograd on the same bf16 weights; relative L2 <= 2e-3 (fp32 accumulation)."""
    from cvlite.fcos_center_net import FCOSCenterNet
    C, B, H, W = 20, 2, 128, 128
    net = FCOSCenterNet(C, seed=0, v1=v1)
    shapes, off, P = net.layout(B, H, W)
    g = torch.Generator().manual_seed(5)
    acts = [_bf(torch.randn(B * P, 256, generator=g, dtype=torch.float64)) for _ in range(2)]
    towers = [[a.to(torch.bfloat16).cuda()] for a in acts]
    reg, cls = net._heads_forward(towers, B, shapes, off, P)
    cc = net.cen_col
    d_cls = torch.zeros((B, P, net.cls_ld), dtype=torch.float64)
    d_cls[..., :C] = torch.randn(B, P, C, generator=g, dtype=torch.float64)
    d_cls[..., cc] = torch.randn(B, P, generator=g, dtype=torch.float64)
    d_reg = torch.zeros((B, P, 32), dtype=torch.float64)
    d_reg[..., :4] = torch.randn(B, P, 4, generator=g, dtype=torch.float64)
    d_cls, d_reg = _bf(d_cls), _bf(d_reg)
    net.store.grad.zero_()
    dA = net._heads_backward((d_reg.to(torch.bfloat16).cuda(), d_cls.to(torch.bfloat16).cuda()),
                             towers, B, shapes, off, P)
    torch.cuda.synchronize()
    # float64 reference
    X = [a.clone().requires_grad_() for a in acts]
    heads = {"cls": net.cls_heads, "cen": net.cen_heads, "reg": net.reg_heads}
    Wt = {k: [_bf(h.w.double().cpu()).requires_grad_() for h in hs] for k, hs in heads.items()}
    Bt = {k: [h.b.double().cpu().requires_grad_() for h in hs] for k, hs in heads.items()}
    total = 0.0
    outs = {"cls": [], "cen": [], "reg": []}
    for l, (h, w) in enumerate(shapes):
        for k, ti, dsl, dst in (("cls", 0, slice(0, C), d_cls), ("cen", 0, slice(cc, cc + 1), d_cls),
                                ("reg", 1, slice(0, 4), d_reg)):
            x = X[ti][B * off[l]:B * off[l] + B * h * w].reshape(B, h, w, 256).permute(0, 3, 1, 2)
            y = torch.nn.functional.conv2d(x, Wt[k][l].permute(3, 2, 0, 1).contiguous(), Bt[k][l], padding=1)
            y = y.permute(0, 2, 3, 1).reshape(B, h * w, -1)
            outs[k].append(y.detach())
            total = total + (y * dst[:, off[l]:off[l] + h * w, dsl]).sum()
    total.backward()
    for l, (h, w) in enumerate(shapes):
        sl = slice(off[l], off[l] + h * w)
        assert _rel(cls[:, sl, :C].double().cpu(), outs["cls"][l]) < 2e-3
        assert _rel(cls[:, sl, cc:cc + 1].double().cpu(), outs["cen"][l]) < 2e-3
        assert _rel(reg[:, sl, :4].double().cpu(), outs["reg"][l]) < 2e-3
        for k, hs in heads.items():
            assert _rel(hs[l].dw.double().cpu(), Wt[k][l].grad) < 2e-3, (k, l)
            assert _rel(hs[l].db.double().cpu(), Bt[k][l].grad) < 2e-3, (k, l)
    assert not cls[..., C:cc].any() and not cls[..., cc + 1:].any() and not reg[..., 4:].any()
    assert _rel(dA[0].double().cpu(), X[0].grad) < 2e-3
    assert _rel(dA[1].double().cpu(), X[1].grad) < 2e-3


@pytest.mark.parametrize("v1", [False, True])
def test_fcos_center_net_train_step(v1):
    """train_fcos_center_voc.py / train_fcos_center_v1_voc.py step on the centre network (graph
    replay): the step's losses equal the oracle's centre model_loss (focal centerness; v1 on the
    sigmoid'd outputs) of the pre-step model's outputs, and the update stays finite."""
    from cvlite.fcos_center_net import FCOSCenterNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    from cvlite import ops_targets as ot
    C, B, D = 20, 2, 128
    net = FCOSCenterNet(C, seed=0, v1=v1)
    tr = FCOSTrainer(net, B, (D, D), targets="center_v1" if v1 else "center")
    imgs, boxes, nbox = synthetic_batch(B, D, D, C, seed=4)
    tr.load_batch(imgs, boxes, nbox)
    if v1:
        tg, _ = ot.fcos_center_v1_assign(tr.boxes, tr.nbox, tr.img_dim, (D, D), C)
    else:
        tg, _ = ot.fcos_center_assign(tr.boxes, tr.nbox, tr.img_dim, (D, D), C, center_only=True)
    reg, cls = net.forward(tr.images)
    nested = [o.cpu().numpy() for o in net.outputs_nested(reg, cls, D, D)]
    shapes, off, P = net.layout(B, D, D)
    tgn = tg.cpu().numpy()
    ref = []
    for b in range(B):
        yt = [tgn[b, off[l]:off[l] + h * w].reshape(h, w, 5 + C) for l, (h, w) in enumerate(shapes)]
        ref.append(fcos_ref.center_model_loss(yt, [o[b:b + 1] for o in nested], cen_type="focal"))
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    assert torch.isfinite(net.store.flat).all()
    tr2 = FCOSTrainer(FCOSCenterNet(C, seed=0, v1=v1), B, (D, D), use_graph=False,
                      targets="center_v1" if v1 else "center")
    tr2.load_batch(imgs, boxes, nbox)
    tr2.step()
    torch.cuda.synchronize()
    np.testing.assert_allclose(tr2.losses.cpu().numpy(), np.array(ref), rtol=1e-4, atol=1e-5)
