"""GPU parity of the RetinaNet anchor matcher, CenterNet centroid targets, centre splat, the
focal + masked smooth-L1 loss and NMS against the reference golden vectors (bit-exact for maps /
indices; losses 2e-5; gradients vs float64 autograd 1e-4)."""
import numpy as np
import pytest
import torch

from oracle import centernet_ref, retina_ref

pytestmark = pytest.mark.gpu


def test_retina_assign_bit_exact(golden):
    from cvlite.retinanet import RetinaNet
    d = golden("retinanet")
    i = 0
    while "case_%d_D" % i in d:
        D = int(d["case_%d_D" % i])
        net = RetinaNet(80, {}, anchor_sizes=list(d["case_%d_sizes" % i]))
        np.testing.assert_array_equal(np.array(net.anchor_boxes, np.float64), d["case_%d_anchor_dims" % i])
        outs, n = net.format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), iou_thresh=0.5, img_pad=[D, D])
        assert n == int(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(np.stack(outs[l]), d["case_%d_L%d" % (i, l)].astype(np.float32))
        i += 1
    assert i >= 10


def test_retina_assign_batched_matches_oracle():
    from cvlite.retinanet import RetinaNet
    rng = np.random.default_rng(9)
    B, D, C, nmax = 4, 640, 80, 50
    net = RetinaNet(C, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = rng.integers(1, nmax + 1, B).astype(np.int32)
    for b in range(B):
        n = nbox[b]
        hw = np.exp(rng.uniform(np.log(8 / D), np.log(0.9), (n, 2)))
        boxes[b, :n, 2:4] = hw
        boxes[b, :n, 0] = rng.uniform(hw[:, 0] / 2, 1 - hw[:, 0] / 2)
        boxes[b, :n, 1] = rng.uniform(hw[:, 1] / 2, 1 - hw[:, 1] / 2)
        boxes[b, :n, 4] = rng.integers(0, C, n)
    dims = np.full((B, 2), D, np.float32)
    tg, nt = net.format_data_batched(torch.tensor(boxes).cuda(), torch.tensor(nbox).cuda(), torch.tensor(dims).cuda(), D)
    tg = tg.cpu().numpy()
    ad = retina_ref.anchor_dims([20.0, 40.0, 80.0, 160.0, 320.0])
    for b in range(B):
        outs, n = retina_ref.format_data(boxes[b, :nbox[b]], dims[b], ad, C, img_pad=[D, D])
        ref = np.concatenate([np.stack(outs[l]).reshape(-1, 4 + C) for l in range(5)], 0)
        np.testing.assert_array_equal(tg[b], ref.astype(np.float32))
        assert int(nt[b]) == n


def test_centernet_assign_and_splat_bit_exact(golden):
    from cvlite import centernet_hourglass as hg
    from cvlite import centernet_splat as cs
    d = golden("centernet")
    for i in range(16):
        D = float(d["hg_%d_D" % i])
        out, n = hg.format_data(d["hg_%d_boxes" % i], np.array([D, D], np.float32), 20, img_pad=[int(D), int(D)],
                                stride=int(d["hg_%d_stride" % i]))
        np.testing.assert_array_equal(out, d["hg_%d_out" % i].astype(np.float32))
        assert n == int(d["hg_%d_n" % i])
    for i in range(12):
        D = float(d["splat_%d_D" % i])
        out = cs.format_data(d["splat_%d_boxes" % i], np.array([D, D], np.float32), 20, img_pad=[int(D), int(D)])
        np.testing.assert_array_equal(out, d["splat_%d_out" % i].astype(np.float32))


def test_centernet_splat_edge_cases():
    from cvlite import centernet_splat as cs
    rng = np.random.default_rng(17)
    for k in range(20):
        D = 512.0
        n = int(rng.integers(1, 30))
        hw = np.exp(rng.uniform(np.log(2 / D), np.log(1.0), (n, 2))).astype(np.float32)
        yc = rng.uniform(hw[:, 0] / 2, 1 - hw[:, 0] / 2)
        xc = rng.uniform(hw[:, 1] / 2, 1 - hw[:, 1] / 2)
        g = np.stack([yc, xc, hw[:, 0], hw[:, 1], rng.integers(0, 20, n)], 1).astype(np.float32)
        area = (g[:, 2] * np.float32(D)) * (g[:, 3] * np.float32(D))
        _, first = np.unique(area, return_index=True)
        g = g[np.sort(first)]
        out = cs.format_data(g, np.array([D, D], np.float32), 20, img_pad=[512, 512])
        np.testing.assert_array_equal(out, centernet_ref.splat_format_data(g, np.array([D, D], np.float32), 20,
                                                                           img_pad=[512, 512]).astype(np.float32))


def test_det_loss_matches_reference_and_grad(golden):
    from cvlite import centernet_hourglass as hg
    from cvlite import ops_targets as ot
    from oracle import fcos_torch
    d = golden("centernet")
    for i in range(6):
        y, p = d["hgloss_%d_y" % i], d["hgloss_%d_p" % i]
        c, r = hg.model_loss(y, p)
        np.testing.assert_allclose([float(c), float(r)], d["hgloss_%d_out" % i], rtol=2e-5)
        C = y.shape[-1] - 4
        t = torch.tensor(y.reshape(1, -1, 4 + C), dtype=torch.float32)
        pp = torch.tensor(p.reshape(1, -1, 4 + C))
        _, dr, dc = ot.det_loss(pp[..., :4].contiguous().cuda(), pp[..., 4:].contiguous().cuda(), t.cuda(), C,
                                grad_scale_cls=2.5, grad_scale_reg=1.0)
        pr = pp[0, :, :4].double().requires_grad_()
        pc = pp[0, :, 4:].double().requires_grad_()
        tt = t[0].double()
        mask = (tt[:, 4:].max(-1).values > 0).double()
        (2.5 * fcos_torch.focal(tt[:, 4:], pc) + fcos_torch.smooth_l1(tt[:, :4], pr, mask)).backward()
        np.testing.assert_allclose(dr[0].cpu().numpy(), pr.grad.numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dc[0].cpu().numpy(), pc.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_nms_matches_reference(golden):
    from cvlite import centernet_hourglass as hg
    d = golden("centernet")
    for i in range(8):
        got = np.array(hg.nms(d["nms_%d_in" % i], 0.213), np.float64).reshape(-1, 6)
        np.testing.assert_array_equal(got, d["nms_%d_out" % i])


def test_soft_nms_and_center_dist_match_reference(golden):
    """cvl_soft_nms vs tf_centernet_hourglass.nms(method='soft-nms') goldens: emission order, boxes
    and classes exact; decayed scores within 4 ulp (the device float64 exp vs numpy's); and
    cvl_center_dist vs tf_centernet.center_dist_1d/2d goldens (float64 pow: 1e-15 relative)."""
    from cvlite import centernet_hourglass as hg
    from cvlite import centernet_splat as cs
    d = golden("centernet_softnms")
    for i in range(8):
        got = np.array(hg.nms(d["soft_%d_in" % i], 0.5, sigma=float(d["soft_%d_sigma" % i]), method="soft-nms"),
                       np.float64).reshape(-1, 6)
        exp = d["soft_%d_out" % i]
        assert got.shape == exp.shape
        np.testing.assert_array_equal(got[:, [0, 1, 2, 3, 5]], exp[:, [0, 1, 2, 3, 5]])
        np.testing.assert_allclose(got[:, 4], exp[:, 4], rtol=1e-15, atol=0)
    c = golden("centernet")
    np.testing.assert_allclose(cs.center_dist_2d(c["cd2_gx"], c["cd2_gy"], 5, 12, 8.0), c["cd2_out"], rtol=1e-15)
    np.testing.assert_allclose(cs.center_dist_1d(np.arange(3, 9) + 0.5, 6, 8.0), c["cd1_out"], rtol=1e-15)


def test_centernet_decode_matches_restatement():
    """cvl_centernet_decode + cvl_nms vs the numpy restatement of obj_detect_results' decode
    (oracle/centernet_ref.py) on random heads: bit-exact rows, including boxes clamped at the image
    border / size limits and an empty result."""
    from cvlite import centernet_hourglass as hg
    rng = np.random.default_rng(11)
    for (H, C, thr, ds, shape) in [(128, 20, 0.5, 4, (500, 375)), (64, 3, 0.3, 8, None), (32, 80, 0.99, 4, None)]:
        pred = np.zeros((H, H, 4 + C), np.float32)
        pred[..., :4] = rng.uniform(-2, 40, size=(H, H, 4)).astype(np.float32)
        pred[..., 4:] = rng.normal(-4.0, 2.5, size=(H, H, C)).astype(np.float32)
        raw, kept = hg.decode_detections(pred, thresh=thr, downsample=ds, img_rows=448, img_cols=448,
                                         img_shape=shape)
        sh = shape or (448, 448)
        ref = centernet_ref.decode_cells(pred, thr, ds, 448, 448, sh[0], sh[1])
        np.testing.assert_array_equal(raw, ref)
        if len(ref):
            np.testing.assert_array_equal(kept, centernet_ref.nms(ref.copy(), 0.213))
    pred = np.full((16, 16, 24), -9.0, np.float32)
    raw, kept = hg.decode_detections(pred)
    assert raw.shape == (0, 6) and kept.shape == (0, 6)


def test_variant_decodes_bit_exact_vs_reference_goldens(golden):
    """cvl_centernet_scale_decode (+ cvl_nms for the s8 form) vs goldens produced by the reference's
    own obj_detect_results (CenterNet/tf_centernet_resnet_s8.py:446-547 and its nms :44-85;
    CenterNet/tf_hourglass_net.py:451-548): bit-exact rows, incl. size clamps and an empty result."""
    from cvlite import tf_centernet_resnet_s8 as s8
    from cvlite import tf_hourglass_net as hg2
    d = golden("variant_decode")
    for i in range(int(d["n_s8"])):
        thr, ds, ir, ic, w, h = d["s8_%d_args" % i]
        raw, kept = s8.decode_detections(d["s8_%d_head" % i], d["s8_%d_scales" % i], thresh=thr, downsample=int(ds),
                                         img_rows=int(ir), img_cols=int(ic), img_shape=(int(w), int(h)))
        np.testing.assert_array_equal(raw, d["s8_%d_raw" % i])
        np.testing.assert_array_equal(kept, d["s8_%d_nms" % i])
    for i in range(int(d["n_hg"])):
        thr, ir, ic, w, h = d["hg_%d_args" % i]
        isc = list(d["hg_%d_scale" % i]) or None
        rows = hg2.decode_detections(torch.from_numpy(d["hg_%d_head" % i]).cuda(), thresh=thr, img_rows=int(ir),
                                     img_cols=int(ic), img_scale=isc, img_shape=(int(w), int(h)))
        np.testing.assert_array_equal(rows, d["hg_%d_rows" % i])
