"""Drop-in semantics of the training-loop API (FCOS/train_fcos.py:87-251,
RetinaNet/train_retinanet_coco.py:145-308) on the GPU path:
* weight_decay > 0: weight_decay * l2_params_reg (sum_v sqrt(sum(l2_loss(v))), computed before the
  tape) enters the reported loss only, not the gradient (train_fcos.py:118-120, 160-171);
* per-image img_dim (the unpadded resized size) reaches format_data with img_pad = the padded
  size (train_fcos.py:131-143);
* train() takes what fcos.build_model returns and the Checkpoint / CheckpointManager pair, and a
  saved checkpoint restores parameters, momentum and BN moving statistics;
* RetinaNet's LR is init for step < 60000 and init / 10 for every later step (:164-171);
* capturing the step graph does not move the BN moving statistics."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_weight_decay_reported_not_differentiated():
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, S = 20, 2, 128
    batch = synthetic_batch(B, S, S, C, seed=5)
    grads, l2s = [], []
    for wd in (0.0, 1e-4):
        net = FCOSNet(C, seed=3)
        p0 = {k: v.double().numpy() for k, v in net.store.state_dict().items()}
        tr = FCOSTrainer(net, B, (S, S), weight_decay=wd)
        tr.load_batch(*batch)
        tr.step()
        torch.cuda.synchronize()
        grads.append(net.store.grad.clone())
        if wd > 0:
            exp = sum(np.sqrt(0.5 * (v ** 2).sum()) for v in p0.values())
            np.testing.assert_allclose(float(tr.l2_params_reg.item()), exp, rtol=1e-5)
    torch.testing.assert_close(grads[1], grads[0], rtol=2e-2, atol=1e-6)


def test_img_dim_per_image_reaches_targets():
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer
    from oracle import fcos_ref
    C, B, S = 20, 2, 384
    net = FCOSNet(C, seed=1)
    tr = FCOSTrainer(net, B, (S, S), use_graph=False)
    rng = np.random.default_rng(3)
    dims = np.array([[300.0, 384.0], [384.0, 257.0]], np.float32)     # resized, unpadded
    boxes = np.zeros((B, 16, 5), np.float32)
    nbox = np.array([5, 7], np.int32)
    for b in range(B):
        for i in range(nbox[b]):
            h, w = np.exp(rng.uniform(np.log(0.05), np.log(0.9), 2))
            boxes[b, i] = [rng.uniform(h / 2, 1 - h / 2), rng.uniform(w / 2, 1 - w / 2), h, w, rng.integers(0, C)]
    imgs = torch.rand((B, S, S, 3), device="cuda") * 2 - 1
    tr.load_batch(imgs, torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), img_dim=torch.from_numpy(dims).cuda())
    tr.step()
    tg = tr.targets.cpu().numpy()
    for b in range(B):
        outs, _ = fcos_ref.format_data(boxes[b, :nbox[b]], dims[b], C, img_pad=(S, S))
        np.testing.assert_array_equal(tg[b], fcos_ref.pack_targets(outs))
    padded, _ = fcos_ref.format_data(boxes[0, :nbox[0]], np.array([S, S], np.float32), C, img_pad=(S, S))
    assert not np.array_equal(tg[0], fcos_ref.pack_targets(padded))       # the unpadded size matters
    tr.load_batch(imgs, torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda())   # back to padded
    tr.step()
    np.testing.assert_array_equal(tr.targets[0].cpu().numpy(), fcos_ref.pack_targets(padded))


def test_train_loop_with_build_model_and_checkpoint_manager(tmp_path, capsys):
    from cvlite import checkpoint as ck
    from cvlite import fcos
    from cvlite.train_fcos import SGD, train
    C, S = 20, 128
    rng = np.random.default_rng(0)
    data = []
    for i in range(6):
        n = int(rng.integers(1, 4))
        hw = rng.uniform(0.1, 0.8, (n, 2))
        c = rng.uniform(hw / 2, 1 - hw / 2)
        data.append(dict(image=rng.uniform(-1, 1, (S, S, 3)).astype(np.float32),
                         bbox=np.concatenate([c, hw], 1).astype(np.float32),
                         label=rng.integers(0, C, n), img_dim=np.array([S, S - 8 * (i % 2)], np.float32)))
    model = fcos.build_model(C)
    opt = SGD(learning_rate=5e-4, momentum=0.9)
    ckpt = ck.Checkpoint(step=ck.Variable(0), fcos_model=model, model_optimizer=opt)
    mgr = ck.CheckpointManager(ckpt, str(tmp_path / "ck"), max_to_keep=1)
    losses = []
    train(data, losses, model, 2, opt, ckpt, mgr, 0, 4, init_lr=5e-4, display_step=2, step_save=2, step_cool=4,
          weight_decay=1e-4, save_loss_file=str(tmp_path / "loss.csv"))
    out = capsys.readouterr().out
    assert "Average Loss:" in out and "Trend Loss:" in out and "Saved model to" in out
    assert int(ckpt.step.numpy()) == 4 and len(losses) == 2 and np.isfinite(losses[-1][1])
    assert mgr.latest_checkpoint.endswith("ckpt-2.pt") and len(mgr.checkpoints) == 1
    # restore into a fresh model: parameters, momentum and moving statistics come back
    net = model.net
    for bn in net.backbone.bns()[:3]:
        assert not torch.equal(bn.run_mean, torch.zeros_like(bn.run_mean))
    model2 = fcos.build_model(C)
    ck2 = ck.Checkpoint(step=ck.Variable(0), fcos_model=model2, model_optimizer=SGD(5e-4, 0.9))
    ck2.restore(mgr.latest_checkpoint)
    assert int(ck2.step.numpy()) == 4
    assert torch.equal(model2.net.store.flat, net.store.flat) and torch.equal(model2.net.store.mom, net.store.mom)
    for a, b in zip(model2.net.backbone.bns(), net.backbone.bns()):
        assert torch.equal(a.run_mean, b.run_mean) and torch.equal(a.run_var, b.run_var)


def test_retinanet_lr_schedule_stays_at_init_over_10():
    from cvlite.retinanet import RetinaNet
    from cvlite.train_retinanet import RetinaTrainer
    from cvlite import ops_nn as nn
    rn = RetinaNet(8, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
    tr = RetinaTrainer(rn.model, rn, 1, 128, n_max=4, init_lr=0.01, min_lr=1e-5, use_graph=False)
    init, mn, rate, dstep = tr.sched
    got = []
    for s in (0, 59999, 60000, 80000, 120000, 500000):
        tr.step_dev.fill_(s)
        nn.lr_schedule(tr.step_dev, tr.lr, init, mn, rate, dstep)
        got.append(float(tr.lr.item()))
    np.testing.assert_allclose(got, [0.01, 0.01, 0.001, 0.001, 0.001, 0.001], rtol=1e-6)


def test_graph_capture_keeps_bn_moving_stats():
    """After the first (captured) step the moving statistics have received exactly one EMA update
    per image, as an eager step gives (the warm-up forwards are undone)."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, B, S = 20, 2, 128
    batch = synthetic_batch(B, S, S, C, seed=9)
    stats = []
    for graph in (False, True):
        net = FCOSNet(C, seed=3)
        tr = FCOSTrainer(net, B, (S, S), use_graph=graph)
        tr.load_batch(*batch)
        tr.step()
        torch.cuda.synchronize()
        stats.append(torch.cat([torch.cat([bn.run_mean, bn.run_var]) for bn in net.backbone.bns()]))
    torch.testing.assert_close(stats[1], stats[0], rtol=1e-4, atol=1e-6)


def _raw_samples(C, seed):
    """Reference-format samples (decoded images, corner boxes, jitter keys) whose jittered padded
    sizes fall in two buckets (256 and 384) with rng seed 11."""
    rng = np.random.default_rng(seed)
    out = []
    for (H, W, lo, hi) in ((150, 180, 150.0, 200.0), (200, 300, 200.0, 250.0), (140, 170, 140.0, 190.0)):
        n = int(rng.integers(1, 5))
        y0, x0 = rng.uniform(0.0, 0.5, n), rng.uniform(0.0, 0.5, n)
        bb = np.stack([y0, x0, y0 + rng.uniform(0.1, 0.5, n), x0 + rng.uniform(0.1, 0.5, n)], -1).astype(np.float32)
        out.append(dict(image=rng.integers(0, 256, (H, W, 3)).astype(np.uint8),
                        objects=dict(bbox=bb, label=rng.integers(0, C, n)), l_jitter=lo, u_jitter=hi,
                        min_side=lo, max_side=1333.0))
    return out


def test_jitter_buckets_sum_gradients_and_update_once():
    """Shape-bucketed FCOS step (train_fcos.py:128-185 per-image jittered sizes): images of a batch
    with different padded sizes run as per-size buckets; the summed gradient and the ONE clip + SGD
    update (1 / batch_size) equal the same buckets run by hand (eager) and summed; preprocess_data's
    boxes equal the reference's flip / swap_xy / convert_to_xywh restatement."""
    from cvlite import ops_nn as nn
    from cvlite.data_preprocess import box_targets, padded_size
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, JitterFCOSTrainer, _raw_batch
    C = 20
    samples = _raw_samples(C, 4)
    imgs, bx, nb, dims = _raw_batch(samples, [0, 1, 2], np.random.default_rng(11))
    sizes = [int(t.shape[0]) for t in imgs]
    assert sorted(set(sizes)) == [256, 384], sizes
    # the host-only size plan draws the same way as preprocess_data
    r2 = np.random.default_rng(11)
    for k, s in enumerate(samples):
        flip, shp, S = padded_size(s["image"].shape[:2], [s["l_jitter"], s["u_jitter"]], s["min_side"],
                                   s["max_side"], r2)
        assert S == sizes[k]
        np.testing.assert_array_equal(dims[k], shp)
        np.testing.assert_array_equal(bx[k, :nb[k], :4], box_targets(s["objects"]["bbox"], flip))
    net = FCOSNet(C, seed=2)
    w0 = net.store.flat.clone()
    jt = JitterFCOSTrainer(net, 3, init_lr=1e-3, use_graph=True)
    losses = jt.step(imgs, bx, nb, dims).cpu()
    torch.cuda.synchronize()
    w_jit = net.store.flat.clone()
    acc_jit = jt.acc.clone()
    assert len(jt.buckets) == 2
    # the same buckets by hand, eager, summed; then the trainer's own update kernels
    ref = FCOSNet(C, seed=2)
    acc = torch.zeros_like(ref.store.grad)
    ref_losses = torch.zeros(3, 3)
    for S in (256, 384):
        idx = [i for i in range(3) if sizes[i] == S]
        tr = FCOSTrainer(ref, len(idx), (S, S), use_graph=False)
        it = torch.tensor(idx)
        tr.load_batch(torch.stack([imgs[i] for i in idx]), torch.from_numpy(bx[idx]).cuda(),
                      torch.from_numpy(nb[idx]).cuda(), img_dim=torch.from_numpy(dims[idx]).cuda())
        tr._fwd_bwd(None)
        acc += ref.store.grad
        ref_losses[it] = tr.losses.cpu()
    torch.testing.assert_close(losses, ref_losses, rtol=1e-5, atol=1e-5)
    e = float((acc_jit - acc).norm() / acc.norm())
    assert e < 1e-5, e
    ref.store.grad.copy_(acc)
    lr = torch.tensor([1e-3], device="cuda")
    nn.sgd_clip_update(ref.store.flat, ref.store.grad, ref.store.mom, lr, 0.9, 1.0 / 3, 1.0,
                       ws=torch.zeros(nn.SUMSQ_WS, dtype=torch.float64, device="cuda"))
    d_ref, d_jit = ref.store.flat - w0, w_jit - w0
    assert float(d_jit.abs().max()) > 0
    assert float((d_jit - d_ref).norm() / d_ref.norm()) < 1e-4


def test_train_loop_raw_samples_jittered(tmp_path):
    """train() on reference-format raw samples: per-image preprocess_data + shape buckets, finite
    losses, weights move."""
    from cvlite import fcos
    from cvlite.train_fcos import SGD, train
    C = 20
    samples = _raw_samples(C, 9) * 2
    from PIL import Image                               # one sample by file name (host decode)
    path = str(tmp_path / "s0.png")
    Image.fromarray(samples[0]["image"]).save(path)
    samples[0] = dict(samples[0], image=path)
    model = fcos.build_model(C)
    net = model.net
    w0 = net.store.flat.clone()
    losses = []
    train(samples, losses, model, 3, SGD(1e-3, 0.9), "", None, 0, 2, display_step=1, step_save=100,
          weight_decay=0.0)
    torch.cuda.synchronize()
    assert torch.isfinite(net.store.flat).all() and not torch.equal(w0, net.store.flat)


def test_train_loop_adam_jittered_checkpoint_roundtrip(tmp_path):
    """train() forwards an Adam optimizer and max_decays into the jitter trainer (Keras Adam is
    what train_fcos_center_voc.py:327 uses); a string ckpt prefix saves the Adam slots and
    load_checkpoint restores them into a fresh trainer."""
    from cvlite import fcos
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_centernet import Adam
    from cvlite.train_fcos import JitterFCOSTrainer, load_checkpoint, train
    C = 20
    samples = _raw_samples(C, 9) * 2
    model = fcos.build_model(C)
    net = model.net
    w0 = net.store.flat.clone()
    opt = Adam(1e-3)
    prefix = str(tmp_path / "adam")
    train(samples, [], model, 3, opt, prefix, None, 0, 2, display_step=1, step_save=2, weight_decay=0.0,
          max_decays=1)
    torch.cuda.synchronize()
    assert int(opt.iterations.item()) == 2
    assert torch.isfinite(net.store.flat).all() and not torch.equal(w0, net.store.flat)
    assert float(opt.v.abs().max()) > 0
    net2 = FCOSNet(C, seed=5)
    opt2 = Adam(1e-3)
    jt = JitterFCOSTrainer(net2, 3, use_graph=False, optimizer=opt2)
    assert load_checkpoint(prefix + ".pt", net2, jt) == 2
    assert torch.equal(net2.store.flat, net.store.flat)
    assert torch.equal(opt2.m, opt.m) and torch.equal(opt2.v, opt.v)
    assert int(opt2.iterations.item()) == 2
