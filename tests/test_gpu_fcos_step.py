"""Whole-step parity of the FCOS trainers (§8a A10: FCOS/train_fcos.py:107-185) and the
round-2 review's variant / boundary fixes.

* FCOSTrainer.step() (HIP-graph replay) twice vs oracle/model_ref.train_step_reference on the same
  device-assigned targets: per-image gradient sum -> /bs -> clip_by_global_norm -> Keras SGD.
* The centre variant trained with Keras Adam (train_fcos_center_voc.py:327) and its step LR
  schedule (:150-157), against the Keras Adam restatement on the trainer's own gradient.
* fcos_center*.build_model(..., "resnet101") builds ResNet-101 (fcos_center.py:37-43).
* JitterFCOSTrainer with a dataset whose busiest image holds more than 16 boxes (a batch without
  that image has narrower box arrays than the bucket trainers).
* split-K vs unsplit accumulation of the same conv launch.
"""
import math

import numpy as np
import pytest
import torch

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu


def _flat_rel(a, b, keys):
    n = d = 0.0
    for k in keys:
        n += float((a[k].double() - b[k].double()).norm() ** 2)
        d += float(b[k].double().norm() ** 2)
    return math.sqrt(n / max(d, 1e-300))


def test_fcos_trainer_two_steps_match_reference_step():
    """Two FCOSTrainer.step() replays at 256x256 / bs 2 (residual-branch gammas damped x0.25 so the
    random-init graph is not chaotic) vs train_step_reference on identical targets.  After each
    step the momentum buffers (= -lr * clipped mean gradient after step 1) and the weight updates
    are compared in rel-L2 over all parameters: bounded by 1.5x the distance bf16 storage alone
    puts between the fp32 oracle and its bf16-storage form, + 0.02."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, D, lr = 20, 2, 256, 5e-4
    net = FCOSNet(C, seed=1)
    for k in net.store.offsets:
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(0.25)
    net.pack()
    p0 = net.store.state_dict()
    tr = FCOSTrainer(net, B, (D, D), init_lr=lr, min_lr=1e-5, use_graph=True)
    imgs, boxes, nbox = synthetic_batch(B, D, D, C, seed=21)
    P16 = {k: v.clone() for k, v in p0.items()}
    P32 = {k: v.clone() for k, v in p0.items()}
    M16 = {k: torch.zeros_like(v) for k, v in p0.items()}
    M32 = {k: torch.zeros_like(v) for k, v in p0.items()}
    names = list(p0)
    for it in range(2):
        tr.load_batch(imgs, boxes, nbox)
        tr.step()
        torch.cuda.synchronize()
        tg = tr.targets.detach().cpu()
        for b in range(B):          # the device targets are the reference's format_data, bit-exact
            outs, _ = fcos_ref.format_data(boxes[b, :int(nbox[b])].cpu().numpy(), np.array([D, D], np.float32), C,
                                           img_pad=(D, D))
            np.testing.assert_array_equal(tg[b].numpy(), fcos_ref.pack_targets(outs))
        x = imgs.cpu()
        with model_ref.emulate_bf16():
            model_ref.train_step_reference(P16, M16, x, tg, C, lr)
        model_ref.train_step_reference(P32, M32, x, tg, C, lr)
        st = net.store
        mom = {k: st.mom[st.offsets[k][0]:st.offsets[k][0] + st.offsets[k][1]].view(st.offsets[k][2]).cpu()
               for k in names}
        dw = {k: net.store.p(k).detach().cpu() - p0[k] for k in names}
        d16 = {k: P16[k] - p0[k] for k in names}
        d32 = {k: P32[k] - p0[k] for k in names}
        own_m, own_w = _flat_rel(M16, M32, names), _flat_rel(d16, d32, names)
        e_m, e_w = _flat_rel(mom, M32, names), _flat_rel(dw, d32, names)
        e_m16, e_w16 = _flat_rel(mom, M16, names), _flat_rel(dw, d16, names)
        print("step %d: momentum rel-L2 gpu-vs-fp32 %.4f gpu-vs-bf16oracle %.4f (bf16 oracle vs fp32 %.4f); "
              "update %.4f / %.4f (%.4f)" % (it + 1, e_m, e_m16, own_m, e_w, e_w16, own_w))
        assert e_m <= 1.5 * own_m + 0.02 and e_m16 <= 1.5 * own_m + 0.02
        assert e_w <= 1.5 * own_w + 0.02 and e_w16 <= 1.5 * own_w + 0.02
    assert int(tr.step_dev.item()) == 2
    assert float(tr.lr.item()) == float(np.float32(lr))       # max(5e-4 * 0.9^floor(1/1000), 1e-5)


def test_fcos_center_trains_with_keras_adam_and_step_schedule():
    """FCOSTrainer(optimizer=Adam) on the centre network: the update equals the Keras Adam
    restatement (oracle/centernet_model_ref.adam_step: divide_no_nan(g, bs), clip_by_global_norm,
    Adam t = iterations + 1) applied to the trainer's own accumulated gradient, at the centre loop's
    learning rate (init_lr below step 8000, init_lr / 10 from step 8000, min_lr floor)."""
    from cvlite.fcos_center_net import FCOSCenterNet
    from cvlite.train_centernet import Adam
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    from oracle import centernet_model_ref as cm
    C, B, D, init_lr = 20, 2, 128, 5e-4
    for st_step, lr in ((0, init_lr), (8000, init_lr / 10.0), (20000, init_lr / 10.0)):
        net = FCOSCenterNet(C, seed=3)
        opt = Adam()
        tr = FCOSTrainer(net, B, (D, D), targets="center", optimizer=opt, init_lr=init_lr, min_lr=1e-6,
                         decay_rate=0.1, decay_step=8000, max_decays=1, st_step=st_step, use_graph=False)
        assert tr.adam is opt and tr.lr is opt.lr_dev
        imgs, boxes, nbox = synthetic_batch(B, D, D, C, seed=9)
        tr.load_batch(imgs, boxes, nbox)
        st = net.store
        names = list(st.offsets)
        p0 = {k: st.p(k).detach().cpu().clone() for k in names}
        tr._fwd_bwd(None)
        torch.cuda.synchronize()
        g = {k: st.g(k).detach().cpu().clone() for k in names}
        tr._update()
        torch.cuda.synchronize()
        assert abs(float(tr.lr.item()) - lr) <= 1e-6 * lr, (st_step, float(tr.lr.item()), lr)
        P = {k: v.clone() for k, v in p0.items()}
        Mo = {k: torch.zeros_like(v) for k, v in P.items()}
        Vo = {k: torch.zeros_like(v) for k, v in P.items()}
        cm.adam_step(P, g, Mo, Vo, 0, lr, B)
        for k in names:
            off, n, shape = st.offsets[k]
            torch.testing.assert_close(st.p(k).detach().cpu(), P[k], rtol=1e-5, atol=1e-7 * max(lr / 1e-4, 1.0))
            torch.testing.assert_close(opt.m[off:off + n].view(shape).cpu(), Mo[k], rtol=1e-5, atol=1e-10)
        assert int(opt.iterations.item()) == 1


@pytest.mark.parametrize("build", ["fcos_center", "fcos_center_v1"])
def test_fcos_center_resnet101_backbone(build):
    """fcos_center.py:37-43 / fcos_center_v1.py:37-43: backbone_model="resnet101" builds ResNet-101
    (conv4_x = 23 blocks, C4 tap conv4_block23_out) -- plain fcos.build_model keeps its
    resnet50-else-MobileNetV2 rule (fcos.py:29-41).  Each ResNet-101 block (conv + per-image BN +
    residual + ReLU) vs the fp32 oracle with the oracle's own input (synced), at 1.5e-2."""
    import torch.nn.functional as F
    from cvlite.fcos_center_net import FCOSCenterNet
    from cvlite.fcos_net import FCOSNet
    from cvlite.mobilenet_v2 import MobileNetV2
    from cvlite.resnet import ResNet50
    assert FCOSNet.backbone_kind("resnet101") == "mobilenetv2"
    C, B, D = 20, 2, 128
    net = FCOSCenterNet(C, backbone_model="resnet101", seed=1, v1=(build == "fcos_center_v1"))
    assert isinstance(net.backbone, ResNet50) and len(net.backbone.stages[2]) == 23
    assert "conv4_block23_3_conv/kernel" in net.store.offsets
    assert isinstance(FCOSCenterNet(C, backbone_model="mobilenetv2", seed=1).backbone, MobileNetV2)
    p = net.store.state_dict()
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.uniform(-1, 1, size=(B, D, D, 3)).astype(np.float32))
    pool, _ = net.backbone.stem.forward(x.cuda())
    xn = x.permute(0, 3, 1, 2)
    hr = F.max_pool2d(F.pad(F.relu(model_ref.bn(model_ref.conv(xn, p, "conv1_conv", 2, pad=3), p, "conv1_bn")),
                            (1, 1, 1, 1)), 3, 2)
    H = W = hr.shape[2]
    for si, stage in enumerate(net.backbone.stages):
        for bi, blk in enumerate(stage):
            n = "conv%d_block%d" % (si + 2, bi + 1)
            s = blk.c1.conv.stride
            hin = hr.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
            out, H, W, _ = blk.forward(hin, B, H, W)
            hb = hin.float().cpu().permute(0, 3, 1, 2)
            sc = model_ref.bn(model_ref.conv(hb, p, n + "_0_conv", s), p, n + "_0_bn") if bi == 0 else hb
            y = F.relu(model_ref.bn(model_ref.conv(hb, p, n + "_1_conv", s), p, n + "_1_bn"))
            y = F.relu(model_ref.bn(model_ref.conv(y, p, n + "_2_conv"), p, n + "_2_bn"))
            hr = F.relu(model_ref.bn(model_ref.conv(y, p, n + "_3_conv"), p, n + "_3_bn") + sc)
            e = float((out.float().cpu().permute(0, 3, 1, 2) - hr).norm() / hr.norm())
            assert e < 1.5e-2, (n, e)
    # the whole centre model runs one training step on the ResNet-101 trunk
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    tr = FCOSTrainer(net, B, (D, D), targets="center_v1" if build == "fcos_center_v1" else "center",
                     use_graph=False)
    tr.load_batch(*synthetic_batch(B, D, D, C, seed=2))
    tr.step()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.losses).all() and torch.isfinite(net.store.flat).all()


def test_jitter_trainer_dataset_with_many_boxes():
    """train()'s raw-sample path sizes the bucket trainers for the busiest image of the dataset
    (here 40 boxes) while a batch without it has box arrays of 16: the bucketed step must pad them
    (and still equal running the same buckets by hand)."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import JitterFCOSTrainer, synthetic_batch
    C, D = 20, 128
    net = FCOSNet(C, seed=0)
    jt = JitterFCOSTrainer(net, 2, n_max=40, use_graph=False)
    imgs, boxes, nbox = synthetic_batch(2, D, D, C, n_max=16, seed=3)
    assert boxes.shape[1] == 16
    losses = jt.step([imgs[0], imgs[1]], boxes, nbox, torch.full((2, 2), float(D)))
    torch.cuda.synchronize()
    assert torch.isfinite(losses).all() and float(losses.sum()) > 0
    tr = next(iter(jt.buckets.values()))
    assert tr.boxes.shape[1] == 40
    assert torch.equal(tr.boxes[:, :16].cpu(), boxes.cpu()) and not tr.boxes[:, 16:].any()


@pytest.mark.parametrize("case", [(2, 8, 8, 256, 256, 3), (2, 16, 16, 128, 128, 3), (4, 8, 8, 512, 512, 3)])
def test_split_k_matches_unsplit(case, dispatch):
    """The split-K accumulation (small grids; CVL_DISPATCH ksplit_min_nk = 4, the default) vs the same launch
    unsplit (ksplit_min_nk huge): fp32 destinations agree to accumulation-order rounding
    (rel-L2 <= 1e-6) and both match the fp64 convolution of the same bf16 operands at 1e-5."""
    import torch.nn.functional as F
    from cvlite import ops_nn as nn
    B, H, W, Cin, Cout, k = case
    g = torch.Generator().manual_seed(H * Cin)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16)
    w = torch.randn(k, k, Cin, Cout, generator=g) * (k * k * Cin) ** -0.5
    npad = (Cout + 31) // 32 * 32
    wf = torch.empty((npad, k * k * Cin), dtype=torch.bfloat16, device="cuda")
    nn.pack_conv_weights(w.cuda().contiguous(), k, k, Cin, Cout, Cin, npad, wf)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), wf.cpu().double()[:Cout].view(Cout, k, k, Cin).permute(0, 3, 1, 2),
                   padding=k // 2).permute(0, 2, 3, 1)
    outs = []
    for min_nk in ("4", "100000"):
        dispatch("ksplit_min_nk=" + min_nk)
        out = torch.zeros((B, H, W, Cout), dtype=torch.float32, device="cuda")
        d = nn.make_desc(nn.FWD, B, Cin, k, k, 1, k // 2, k // 2, npad, Cout, Cout, [nn.seg(H, W, H, W, wf, None)],
                         dst_f32=True)
        nn.conv_igemm(d, x.cuda(), out)
        torch.cuda.synchronize()
        outs.append(out.double().cpu())
    e_split = float((outs[0] - outs[1]).norm() / outs[1].norm())
    print("split vs unsplit rel-L2 %.2e (bit-identical: %s)" % (e_split, torch.equal(outs[0], outs[1])))
    assert e_split <= 1e-6
    for o in outs:
        assert float((o - ref).norm() / ref.norm()) <= 1e-5


def test_tower0_dgrad_forms_agree(dispatch):
    """Tower layer 0's two data gradients (both towers read the shared F): the paired launch into a
    temporary + one add (default) and two launches accumulating into dF
    (CVL_DISPATCH=no_tower0_pair) give dF within bf16 rounding, and the whole trunk backward agrees."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import synthetic_batch
    C, B, D = 20, 2, 128
    res = {}
    for flag in ("1", "0"):
        dispatch("no_tower0_pair=" + ("0" if flag == "1" else "1"))
        net = FCOSNet(C, seed=5)
        imgs, _, _ = synthetic_batch(B, D, D, C, seed=1)
        reg, cls = net.forward(imgs)
        P = reg.shape[1]
        g = torch.Generator().manual_seed(2)
        d_reg = (torch.randn((B, P, 32), generator=g) * 0.1).to(torch.bfloat16).cuda()
        d_cls = (torch.randn((B, P, net.cls_ld), generator=g) * 0.1).to(torch.bfloat16).cuda()
        d_reg[..., 5:] = 0
        d_cls[..., C:] = 0
        net.backward(d_reg, d_cls)
        torch.cuda.synchronize()
        res[flag] = {k: net.store.g(k).detach().cpu().clone() for k in net.store.offsets}
    keys = [k for k in res["1"] if float(res["1"][k].norm()) > 0]
    e = _flat_rel(res["0"], res["1"], keys)
    print("tower-0 paired vs accumulate: gradient rel-L2 %.2e" % e)
    assert e < 2e-2
    for k in ("cls_layer_1/kernel", "reg_layer_1/kernel", "c3_3x3/kernel"):
        assert float((res["0"][k] - res["1"][k]).norm() / res["1"][k].norm()) < 2e-2, k


@pytest.mark.parametrize("exact", [True, False])
def test_fcos_step_run_to_run_bit_identical(exact):
    """Reproducibility: two trainers built from the same seed run two graph-replayed
    steps on the same 512x512 batch and end with bit-identical parameters, momentum buffers and
    losses.  The split reductions (weight-gradient slabs, split-K, gradient norm) sum in a fixed
    order.  The fused BN statistics: in the exact mode (cvl_bn_set_exact) integer bins, identical by
    construction; in the default mode fp64 atomics of fp32 partials, which can differ in the last
    bits only when a statistic's partials span more than fp64's 53 bits -- observed identical here."""
    from cvlite import ops_nn as nn
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    nn.set_bn_exact(exact)
    try:
        _run_to_run(exact)
    finally:
        nn.set_bn_exact(False)


def _run_to_run(exact):
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, D = 20, 4, 512
    imgs, boxes, nbox = synthetic_batch(B, D, D, C, seed=7)
    res = []
    for _ in range(2):
        net = FCOSNet(C, seed=3)
        tr = FCOSTrainer(net, B, (D, D), use_graph=True)
        tr.load_batch(imgs, boxes, nbox)
        tr.step()
        tr.load_batch(imgs, boxes, nbox)
        tr.step()
        torch.cuda.synchronize()
        res.append((net.store.flat.clone(), net.store.mom.clone(), tr.losses.clone()))
        del tr, net
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
