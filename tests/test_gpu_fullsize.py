"""Whole training steps at the BASELINE.json configurations, on the production dispatch (HIP
graphs, no knobs): configs[1] FCOS R50-FPN 512x512 bs 16, configs[3] CenterNet hourglass
512x512 bs 8, configs[4] RetinaNet R50-FPN 640x640 bs 8 C = 80 (3*bs candidates).

Each asserts, on that step's own batch:
* the device targets are bit-exact vs the oracle restatement (oracle/*_ref.py, pinned to the
  reference's own functions by tests/golden/make_golden.py);
* the per-image losses the fused loss kernel reported equal the oracle loss evaluated on the
  GPU's own head outputs (rtol 2e-5: fp32 sums of ~10^5 terms in a different order);
* the update produced finite weights that moved.
RetinaNet additionally checks cvl_retina_loss's gradient against float64 autograd on a 1-image
slice of that batch (C = 80, all 76,725 anchors)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _finite_and_moved(store, w0):
    torch.cuda.synchronize()
    assert torch.isfinite(store.flat).all() and torch.isfinite(store.grad).all()
    assert float((store.flat - w0).abs().max()) > 0


def test_fcos_step_configs1():
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    from oracle import fcos_ref
    C, B, S = 20, 16, 512
    net = FCOSNet(C, seed=0)
    tr = FCOSTrainer(net, B, (S, S))
    imgs, boxes, nbox = synthetic_batch(B, S, S, C, seed=2024)
    tr.load_batch(imgs, boxes, nbox)
    w0 = net.store.flat.clone()
    losses = tr.step().clone()
    _finite_and_moved(net.store, w0)
    tg = tr.targets.cpu().numpy()
    reg, cls = (t.cpu().numpy() for t in tr.outputs)
    bx, nb = boxes.cpu().numpy(), nbox.cpu().numpy()
    sizes = [64, 32, 16, 8, 4]
    got = losses.cpu().double().numpy()
    for b in range(B):
        outs, _ = fcos_ref.format_data(bx[b, :nb[b]], np.array([S, S], np.float32), C, img_pad=(S, S))
        np.testing.assert_array_equal(tg[b], fcos_ref.pack_targets(outs))
        pred = np.concatenate([reg[b, :, :5], cls[b, :, :C]], 1)
        preds, o = [], 0
        for s in sizes:
            preds.append(pred[o:o + s * s].reshape(1, s, s, 5 + C))
            o += s * s
        ref = np.array(fcos_ref.model_loss(outs, preds), np.float64)
        np.testing.assert_allclose(got[b], ref, rtol=2e-5, atol=1e-4)
    # a second replayed step on another batch stays finite and keeps training
    tr.load_batch(*synthetic_batch(B, S, S, C, seed=2025))
    assert torch.isfinite(tr.step()).all()


def test_centernet_step_configs3():
    from cvlite.hourglass_net import HourglassNet
    from cvlite.train_centernet import CenterNetTrainer, synthetic_batch
    from oracle import centernet_ref
    C, B, S = 20, 8, 512
    net = HourglassNet(C, seed=0)
    tr = CenterNetTrainer(net, B, (S, S), sub_batch_sz=2, n_max=16)
    imgs, boxes, nbox = synthetic_batch(B, S, S, C, n_max=16, seed=77)
    tr.load_batch(imgs, boxes, nbox)
    w0 = net.store.flat.clone()
    losses = tr.step().clone()
    _finite_and_moved(net.store, w0)
    tg = tr.targets.cpu().numpy()
    out = tr.out.cpu().numpy()
    bx, nb = boxes.cpu().numpy(), nbox.cpu().numpy()
    got = losses.cpu().double().numpy()
    assert tr.stride == 4 and tg.shape[1:3] == (128, 128)
    for b in range(B):
        ref, n = centernet_ref.hourglass_format_data(bx[b, :nb[b]], np.array([S, S], np.float32), C,
                                                     img_pad=[S, S], stride=tr.stride)
        np.testing.assert_array_equal(tg[b], ref.astype(np.float32))
        pred = out[b][..., :4 + C]
        rc, rr = centernet_ref.hourglass_model_loss(ref.astype(np.float32), pred)
        np.testing.assert_allclose(got[b], [rc, rr], rtol=2e-5, atol=1e-4)


def test_retinanet_step_configs4():
    from cvlite import ops_targets as ot
    from cvlite.retinanet import RetinaNet
    from cvlite.train_retinanet import RetinaTrainer, synthetic_coco_batch
    from oracle import fcos_torch, model_ref, retina_ref
    C, A, B, S = 80, 9, 8, 640
    sizes = [20.0, 40.0, 80.0, 160.0, 320.0]
    rn = RetinaNet(C, {}, anchor_sizes=sizes)
    net = rn.model
    tr = RetinaTrainer(net, rn, B, S, n_max=50)
    imgs, boxes, nbox = synthetic_coco_batch(3 * B, S, C, n_max=50, seed=4321)
    tr.load_candidates(imgs, boxes, nbox)
    w0 = net.store.flat.clone()
    losses = tr.step().clone()
    _finite_and_moved(net.store, w0)
    # targets of all 3*bs candidates, bit-exact, and the reference's selection rule
    ad = retina_ref.anchor_dims(sizes)
    ctg = tr.cand_targets.cpu().numpy()
    cnt = tr.cand_counts.cpu().numpy()
    bx, nb = boxes.cpu().numpy(), nbox.cpu().numpy()
    for i in range(3 * B):
        outs, n = retina_ref.format_data(bx[i, :nb[i]], np.array([S, S], np.float32), ad, C, img_pad=[S, S])
        ref = np.concatenate([np.stack(outs[l]).reshape(-1, 4 + C) for l in range(5)], 0)
        np.testing.assert_array_equal(ctg[i], ref.astype(np.float32))
        assert int(cnt[i]) == n
    exp_sel = [i for i in range(3 * B) if cnt[i] > 0][:B]
    assert tr.sel.cpu().tolist()[:len(exp_sel)] == exp_sel
    # per-image losses vs the oracle on the GPU's own head outputs
    reg, cls = tr.outputs
    cells = tr.level_cells
    P = sum(cells)
    t = model_ref.retina_unpack_targets(tr.targets.cpu().double(), cells, A)         # [B, P, A, 4+C]
    w = tr.img_w.cpu().numpy()
    got = losses.cpu().double().numpy()
    rr_all = reg.cpu().double()[..., :4 * A].reshape(B, P, A, 4)
    cc_all = cls.cpu().double()[..., :A * C].reshape(B, P, A, C)
    for b in range(B):
        tb = t[b].reshape(P * A, 4 + C)
        mask = (tb[:, 4:].max(-1).values > 0).double()
        lc = float(fcos_torch.focal(tb[:, 4:], cc_all[b].reshape(P * A, C)))
        lr = float(fcos_torch.smooth_l1(tb[:, :4], rr_all[b].reshape(P * A, 4), mask))
        np.testing.assert_allclose(got[b], [lc * w[b], lr * w[b]], rtol=2e-5, atol=1e-3)
    # cvl_retina_loss gradient vs float64 autograd on image 0 of that batch
    d_reg = torch.zeros((1, P, net.reg_ld), dtype=torch.bfloat16, device="cuda")
    d_cls = torch.zeros((1, P, net.cls_ld), dtype=torch.bfloat16, device="cuda")
    ot.retina_loss(reg[:1].contiguous(), cls[:1].contiguous(), tr.targets[:1].contiguous(), cells, A, C,
                   grad_scale=1.0, d_reg=d_reg, d_cls=d_cls)
    r0 = rr_all[0].clone().requires_grad_(True)
    c0 = cc_all[0].clone().requires_grad_(True)
    tb = t[0]
    mask = (tb[..., 4:].max(-1).values > 0).double()
    (fcos_torch.focal(tb[..., 4:], c0) + fcos_torch.smooth_l1(tb[..., :4], r0, mask)).backward()
    gr = d_reg.double().cpu()[0, :, :4 * A].reshape(P, A, 4)
    gc = d_cls.double().cpu()[0, :, :A * C].reshape(P, A, C)
    bad = ((gc - c0.grad).abs() > 1e-3 + 1e-2 * c0.grad.abs()).nonzero()
    for (p_, a_, c_) in bad[:8].tolist():
        print("mismatch cell %d anchor %d class %d: logit %r target %r kernel %r autograd %r" % (
            p_, a_, c_, float(c0[p_, a_, c_]), float(tb[p_, a_, 4 + c_]), float(gc[p_, a_, c_]),
            float(c0.grad[p_, a_, c_])))
    torch.testing.assert_close(gr, r0.grad, rtol=1e-2, atol=1e-2)       # bf16 gradient storage
    torch.testing.assert_close(gc, c0.grad, rtol=1e-2, atol=1e-3)
    assert torch.count_nonzero(d_cls[..., A * C:]).item() == 0
