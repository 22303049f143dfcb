"""Pin the CPU oracle (oracle/*.py) to golden vectors produced by the reference's own functions
(tests/golden/make_golden.py).  Bit-exact for targets / indices / anchors; 1e-6 relative for
float losses (the goldens were computed with fp32 numpy elementwise ops, the oracle in float64)."""
import json

import numpy as np
import pytest

from oracle import centernet_ref, fcos_ref, retina_ref


def test_fcos_format_data_bit_exact(golden):
    d = golden("fcos")
    meta = json.loads(str(d["meta"]))
    branches = 0
    for i in range(meta["n_images"]):
        outs, nt = fcos_ref.format_data(d["assign_%d_boxes" % i], d["assign_%d_img_dim" % i],
                                        meta["C"], img_pad=tuple(int(x) for x in d["assign_%d_img_pad" % i]))
        assert list(nt) == list(d["assign_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(outs[l], d["assign_%d_L%d" % (i, l)])
        branches += sum(int(o[..., 5:].sum() > 0) for o in outs)
    assert branches > 40


def test_fcos_losses(golden):
    d = golden("fcos")
    meta = json.loads(str(d["meta"]))
    for i in meta["loss_imgs"]:
        tgt = [d["assign_%d_L%d" % (i, l)] for l in range(5)]
        pr = [d["loss_%d_pred_L%d" % (i, l)] for l in range(5)]
        for rt in ("l1", "iou"):
            np.testing.assert_allclose(fcos_ref.model_loss(tgt, pr, reg_type=rt), d["loss_%d_%s" % (i, rt)],
                                       rtol=1e-6)
    np.testing.assert_allclose(fcos_ref.focal_loss(d["focal_y"], d["focal_x"]), d["focal_out"], rtol=1e-6)
    np.testing.assert_allclose(fcos_ref.smooth_l1_loss(d["sl1_true"], d["sl1_pred"], d["sl1_mask"]),
                               d["sl1_out"], rtol=1e-6)
    np.testing.assert_allclose(fcos_ref.smooth_l1_loss(d["sl1_true"], d["sl1_pred"]), d["sl1_out_nomask"],
                               rtol=1e-6)
    np.testing.assert_array_equal(fcos_ref.prediction_to_corners(d["p2c_in"], 16), d["p2c_out"])


def test_loss_keyword_surface(golden):
    """focal_loss(alpha, gamma) / smooth_l1_loss(mask, delta) at non-default keywords and soft
    labels / masks (goldens from the reference's own functions)."""
    d = golden("loss_kwargs")
    meta = json.loads(str(d["meta"]))
    for k, (alpha, gamma) in enumerate(meta["focal"]):
        np.testing.assert_allclose(fcos_ref.focal_loss(d["focal_%d_y" % k], d["focal_%d_x" % k], alpha, gamma),
                                   d["focal_%d_out" % k], rtol=1e-6)
    for k, (delta, kind) in enumerate(meta["sl1"]):
        m = d["sl1_%d_mask" % k] if kind != "none" else 1.0
        np.testing.assert_allclose(fcos_ref.smooth_l1_loss(d["sl1_%d_true" % k], d["sl1_%d_pred" % k], m, delta),
                                   d["sl1_%d_out" % k], rtol=1e-6)


def test_retinanet_anchor_and_match_bit_exact(golden):
    d = golden("retinanet")
    i = 0
    while "case_%d_D" % i in d:
        D = int(d["case_%d_D" % i])
        dims = retina_ref.anchor_dims(list(d["case_%d_sizes" % i]))
        np.testing.assert_array_equal(dims.astype(np.float64), d["case_%d_anchor_dims" % i])
        outs, n = retina_ref.format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), dims, 80,
                                         img_pad=[D, D])
        assert n == int(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(np.stack(outs[l]), d["case_%d_L%d" % (i, l)])
        i += 1
    assert i >= 10
    dims = retina_ref.anchor_dims([20.0, 40.0, 80.0, 160.0, 320.0])
    np.testing.assert_array_equal(np.stack(retina_ref.get_anchors(dims, [5, 5], 4)), d["get_anchors_5x5_L4"])
    np.testing.assert_array_equal(retina_ref.compute_iou(d["iou_b1"], d["iou_b2"]), d["iou_out"])


def test_centernet_targets_splat_nms(golden):
    d = golden("centernet")
    for i in range(16):
        D = float(d["hg_%d_D" % i])
        o, n = centernet_ref.hourglass_format_data(d["hg_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                                   img_pad=[int(D), int(D)], stride=int(d["hg_%d_stride" % i]))
        np.testing.assert_array_equal(o, d["hg_%d_out" % i])
        assert n == int(d["hg_%d_n" % i])
    for i in range(6):
        np.testing.assert_allclose(centernet_ref.hourglass_model_loss(d["hgloss_%d_y" % i], d["hgloss_%d_p" % i]),
                                   d["hgloss_%d_out" % i], rtol=1e-6)
    for i in range(12):
        D = float(d["splat_%d_D" % i])
        o = centernet_ref.splat_format_data(d["splat_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                            img_pad=[int(D), int(D)])
        np.testing.assert_array_equal(o, d["splat_%d_out" % i])
    np.testing.assert_array_equal(centernet_ref.center_dist_2d(d["cd2_gx"], d["cd2_gy"], 5, 12, 8.0), d["cd2_out"])
    np.testing.assert_array_equal(centernet_ref.center_dist_1d(np.arange(3, 9) + 0.5, 6, 8.0), d["cd1_out"])
    for i in range(8):
        np.testing.assert_array_equal(centernet_ref.nms(d["nms_%d_in" % i], 0.213), d["nms_%d_out" % i])


def _retina_decode_case(d, i):
    D, C, iou_t, cls_t = d["case_%d_cfg" % i]
    dims = d["case_%d_anchor_dims" % i]
    outs = [list(d["case_%d_out_L%d" % (i, l)]) for l in range(5)]
    return int(D), int(C), float(iou_t), float(cls_t), dims, outs


def test_retina_decode_nms_oracle(golden):
    """retinanet_module.py:428-529: corners bit-exact, cpu_nms indices exact, image_detections
    rows: boxes/labels exact, scores within 4 fp32 ulp (sigmoid evaluation order)."""
    d = golden("retina_decode")
    np.testing.assert_array_equal(retina_ref.prediction_to_corners(d["corners_in"], d["corners_dims"], 32),
                                  d["corners_out"])
    np.testing.assert_array_equal(retina_ref.cpu_nms(d["nms_dets"], 0.45), d["nms_keep"])
    i = 0
    while "case_%d_cfg" % i in d:
        D, C, iou_t, cls_t, dims, outs = _retina_decode_case(d, i)
        got = retina_ref.image_detections(outs, dims, iou_thresh=iou_t, cls_thresh=cls_t)
        ref = d["case_%d_dets" % i]
        assert got.shape == ref.shape
        np.testing.assert_array_equal(got[:, [0, 1, 2, 3, 5]], ref[:, [0, 1, 2, 3, 5]])
        np.testing.assert_allclose(got[:, 4], ref[:, 4], rtol=5e-7, atol=0)
        i += 1
    assert i == 4


def test_fcos_combined_nms_known_answer():
    """Hand-worked case of the tf.image.combined_non_max_suppression restatement (TF is absent:
    this pins the published semantics, not TF itself): score > threshold (strict), per-class
    greedy with IoU > thr suppressing, degenerate boxes never suppress, per-class cap, merge by
    descending score, zero padding, valid count."""
    boxes = np.array([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [5, 5, 5, 9], [0, 0, 10, 10]], np.float32)
    scores = np.array([[0.9, 0.1], [0.8, 0.7], [0.3, 0.05], [0.6, 0.2], [0.05, 0.95]], np.float32)
    b, s, c, n = fcos_ref.combined_non_max_suppression(boxes, scores, 2, 6, iou_threshold=0.5, score_threshold=0.05)
    # class 0: 0 (0.9) keeps; 1 (0.8) IoU 81/119 > 0.5 suppressed; 3 (0.6, zero area) kept -> cap 2 reached
    # class 1: 4 (0.95); 1 (0.7) IoU with 4 = 81/119 suppressed; 3 (0.2) kept; 2 (0.05) not > 0.05
    assert n == 4
    np.testing.assert_array_equal(s, np.array([0.95, 0.9, 0.6, 0.2, 0, 0], np.float32))
    np.testing.assert_array_equal(c, np.array([1, 0, 0, 1, 0, 0], np.float32))
    np.testing.assert_array_equal(b[:4], boxes[[4, 0, 3, 3]])
    assert not b[4:].any()


def test_preprocess_resize_known_answers():
    """TF2 bilinear resize restatement (data_preprocess.py:41-96; TF absent): equal size is the
    identity, an exact 2x downscale is the mean of each 2x2 block, edges clamp."""
    from oracle import preprocess_ref as pr
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (6, 8, 3)).astype(np.float32)
    np.testing.assert_array_equal(pr.resize_bilinear(a, 6, 8), a)
    d = pr.resize_bilinear(a, 3, 4)
    blocks = a.reshape(3, 2, 4, 2, 3).mean(axis=(1, 3))
    np.testing.assert_allclose(d, blocks, rtol=0, atol=1e-4)
    up = pr.resize_bilinear(a[:1, :1], 3, 3)
    assert (up == a[0, 0]).all()
    img, ns, r = pr.resize_and_pad_image(a.astype(np.uint8), 12.0, 100.0, 8.0, True)
    assert img.shape == (16, 16, 3) and tuple(ns) == (12.0, 16.0) and r == np.float32(2.0)
    assert not img[12:].any()


def _center_cases(d):
    i = 0
    while "case_%d_cfg" % i in d:
        D, co = (int(v) for v in d["case_%d_cfg" % i])
        yield i, D, bool(co)
        i += 1


def test_fcos_center_format_data_bit_exact(golden):
    """FCOS/fcos_center.py:149-317 restatement vs the reference's own outputs."""
    d = golden("fcos_center")
    overlaps = 0
    for i, D, co in _center_cases(d):
        outs, nt = fcos_ref.center_format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                               img_pad=[D, D], center_only=co)
        assert list(nt) == list(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(outs[l].astype(np.float32), d["case_%d_L%d" % (i, l)])
            overlaps += int((d["case_%d_L%d" % (i, l)][..., 5:].sum(-1) > 1).sum())
    assert overlaps > 0


def test_centernet_soft_nms_oracle(golden):
    """tf_centernet_hourglass.nms(method='soft-nms') goldens (make_golden.py centernet_softnms):
    emission order and boxes exact, decayed scores bit-exact (same float64 numpy sequence)."""
    d = golden("centernet_softnms")
    for i in range(8):
        got = centernet_ref.soft_nms(d["soft_%d_in" % i], float(d["soft_%d_sigma" % i]))
        np.testing.assert_array_equal(got, d["soft_%d_out" % i])


def test_fcos_center_v1_format_data_and_losses(golden):
    """FCOS/fcos_center_v1.py format_data (bit-exact maps and counts) and model_loss (the v1 model's
    sigmoid reg head), and fcos_center.py model_loss with cen_type="focal", vs the reference's own
    outputs (make_golden.py fcos_center_v1)."""
    d = golden("fcos_center_v1")
    n_loss = 0
    for i in range(16):
        D = int(d["case_%d_D" % i])
        outs, nt = fcos_ref.center_v1_format_data(d["case_%d_boxes" % i], np.array([D, D], np.float32), 20,
                                                  img_pad=[D, D])
        assert list(nt) == list(d["case_%d_ntgt" % i])
        for l in range(5):
            np.testing.assert_array_equal(outs[l].astype(np.float32), d["case_%d_L%d" % (i, l)])
        if "loss_%d_out" % i in d.files:
            n_loss += 1
            yt = [d["case_%d_L%d" % (i, l)] for l in range(5)]
            raw = [d["loss_%d_raw_L%d" % (i, l)] for l in range(5)]
            np.testing.assert_allclose(fcos_ref.center_model_loss(yt, raw, cen_type="focal", reg_sigmoid=True),
                                       d["loss_%d_out" % i], rtol=1e-5)
            np.testing.assert_allclose(fcos_ref.center_model_loss(yt, raw, cen_type="focal"),
                                       d["loss_%d_center_focal" % i], rtol=1e-5)
    assert n_loss == 3
    np.testing.assert_array_equal(fcos_ref.center_v1_prediction_to_corners(d["p2c_in"], 320.0, 16), d["p2c_out"])


def test_hourglass_v2_targets_and_loss(golden):
    """CenterNet v2: the restated target builder vs the maps the reference's own
    train_hourglass_voc.train() built (bit-exact), and model_loss (focal / sigmoid) vs the
    reference's tf_hourglass_net.model_loss (rtol 1e-5: fp32 TF ops vs the float64 restatement)."""
    from oracle import hourglass_v2_ref as hv
    d = golden("hourglass_v2")
    C = int(d["C"])
    n_rows = 0
    for st in range(6):
        raw, img = (int(v) for v in d["step_%d_raw_img" % st])
        got = hv.format_data(d["step_%d_boxes" % st], d["step_%d_nbox" % st], raw, img, C)
        np.testing.assert_array_equal(got, d["step_%d_targets" % st])
        n_rows += int((got[..., 4] > 0).sum())
    assert n_rows > 200
    for st in (0, 3):
        t = d["loss_%d_targets" % st]
        for lt in ("focal", "sigmoid"):
            np.testing.assert_allclose(hv.model_loss(t, d["loss_%d_raw" % st], d["loss_%d_bfocal" % st], lt),
                                       d["loss_%d_%s" % (st, lt)], rtol=1e-5)


def test_centernet_s8_targets_and_loss(golden):
    """tf_centernet_resnet_s8.format_data (float64 rows as the crowdhuman trainer feeds it) and
    model_loss vs the reference's own outputs."""
    from oracle import centernet_s8_ref as s8
    d = golden("centernet_s8")
    scales = [32.0, 64.0, 128.0, 256.0, 512.0]
    hits = 0
    for i in range(12):
        raw, img = (int(v) for v in d["case_%d_dims" % i])
        out, n = s8.format_data(d["case_%d_rows" % i], scales, [raw, raw], 3, img_pad=[img, img])
        np.testing.assert_array_equal(out, d["case_%d_out" % i])
        assert n == int(d["case_%d_n" % i])
        hits += int((out[..., 4:].sum(-1) > 0).sum())
    assert hits > 100
    pred = np.concatenate([1.0 / (1.0 + np.exp(-d["loss_reg_logits"].astype(np.float64))), d["loss_cls_logits"]], -1)
    np.testing.assert_allclose(s8.model_loss(d["loss_y"], pred), d["loss_out"], rtol=1e-5)


def test_centernet_peak_decode_restatement_known_answer():
    """oracle/centernet_peak_ref.py on a hand-made 5x5, 2-class map: local maxima only (3x3, ties on a
    plateau all kept), threshold, probability-descending order with flat-index tie break, K cut,
    prediction_to_corners boxes (tf_centernet_hourglass.py:355-377).  No reference implementation
    exists (the reference decodes by threshold + NMS): parity unpinned at the reference level."""
    import numpy as np
    from oracle.centernet_peak_ref import peak_decode
    H, W, C = 5, 5, 2
    pred = np.zeros((H, W, 4 + C), np.float32)
    pred[..., :4] = [1.0, 2.0, 3.0, 4.0]                    # (top, bottom, left, right) in cells
    cls0 = np.full((H, W), -6.0, np.float32)
    cls0[1, 1] = 2.0                                         # isolated peak
    cls0[1, 2] = 1.0                                         # its neighbour: suppressed
    cls0[3, 3] = cls0[3, 4] = 0.5                            # plateau: both kept
    cls0[4, 0] = -3.0                                        # a local max below thresh
    cls1 = np.full((H, W), -6.0, np.float32)
    cls1[1, 1] = 2.0                                         # same prob as class 0 at (1,1)
    pred[..., 4], pred[..., 5] = cls0, cls1
    rows = peak_decode(pred, C, stride=8, thresh=0.3, K=10)
    # order: (1,1) c0 [idx 12], (1,1) c1 [idx 13], then the plateau (3,3) [36], (3,4) [38]
    assert rows.shape == (4, 6)
    np.testing.assert_array_equal(rows[:, 5], [0, 1, 0, 0])
    np.testing.assert_allclose(rows[0, :4], [8 * (1.5 - 1), 8 * (1.5 - 3), 8 * (1.5 + 2), 8 * (1.5 + 4)])
    np.testing.assert_allclose(rows[2, :4], [8 * (3.5 - 1), 8 * (3.5 - 3), 8 * (3.5 + 2), 8 * (3.5 + 4)])
    np.testing.assert_allclose(rows[3, :4], [8 * (3.5 - 1), 8 * (4.5 - 3), 8 * (3.5 + 2), 8 * (4.5 + 4)])
    np.testing.assert_allclose(rows[:, 4], 1 / (1 + np.exp(-np.array([2.0, 2.0, 0.5, 0.5]))), rtol=1e-6)
    assert len(peak_decode(pred, C, 8, 0.3, K=1)) == 1
    assert len(peak_decode(pred, C, 8, 0.99, K=10)) == 0


def test_image_augment_restatement_vs_reference(golden):
    """oracle/augment_ref.py vs the reference's own image_augment (train_hourglass_voc.py:24-67, run by
    make_golden.py): with the same numpy seed the restated draws take the same branch, and the
    transformed image and float64 target map are bit-identical (all six branches occur)."""
    from oracle import augment_ref as A
    z = golden("image_augment")
    seen = set()
    for k in range(int(z["n_cases"])):
        sn, st = (int(v) for v in z["case_%d_seeds" % k])
        op, prm = A.draw_augment(rng=np.random.RandomState(sn), tf_rng=np.random.RandomState(st))
        seen.add(op)
        im, bb = A.image_augment_ref(z["case_%d_img" % k], z["case_%d_bbox" % k], op, prm)
        assert np.array_equal(im, z["case_%d_out_img" % k]), (k, op)
        assert np.array_equal(bb, z["case_%d_out_bbox" % k]), (k, op)
    assert seen == set(range(6)), seen


def test_image_augment_product_draws_match_restatement():
    """cvlite.train_hourglass_v2.draw_augment consumes the numpy stream exactly as the reference's
    image_augment does (same branch, same state afterwards) over many seeds."""
    from oracle import augment_ref as A
    from cvlite.train_hourglass_v2 import draw_augment
    for s in range(300):
        r1, r2 = np.random.RandomState(s), np.random.RandomState(s)
        t1, t2 = np.random.RandomState(s + 7), np.random.RandomState(s + 7)
        assert draw_augment(0.5, rng=r1, tf_rng=t1) == A.draw_augment(0.5, rng=r2, tf_rng=t2)
        assert r1.uniform() == r2.uniform()


def _hg2_box_scales(ir, ic, isc):
    if not len(isc):
        isc = [64, 128, 256, max(ir, ic) if max(ir, ic) < 512 else 512]
    return list(isc[:3]) + [max(ir, ic) if max(ir, ic) <= isc[3] else isc[3]]


def test_variant_decode_oracle(golden):
    """The variant CenterNets' obj_detect_results decodes (tf_centernet_resnet_s8.py:446-547 incl. its
    nms; tf_hourglass_net.py:451-548): the restatements vs goldens produced by the reference's own
    functions (plotting recorded, not drawn) -- bit-exact rows, incl. size clamps and an empty case."""
    d = golden("variant_decode")
    for i in range(int(d["n_s8"])):
        thr, ds, ir, ic, w, h = d["s8_%d_args" % i]
        raw = centernet_ref.decode_s8_cells(d["s8_%d_head" % i], d["s8_%d_scales" % i], thr, int(ds), int(ir),
                                            int(ic), int(w), int(h))
        np.testing.assert_array_equal(raw, d["s8_%d_raw" % i])
        if len(raw):
            np.testing.assert_array_equal(np.array(centernet_ref.nms(raw.copy(), 0.213)).reshape(-1, 6),
                                          d["s8_%d_nms" % i])
    for i in range(int(d["n_hg"])):
        thr, ir, ic, w, h = d["hg_%d_args" % i]
        bs = _hg2_box_scales(int(ir), int(ic), list(d["hg_%d_scale" % i]))
        rows = centernet_ref.decode_hg2_cells(d["hg_%d_head" % i], thr, int(ir), int(ic), bs, int(w), int(h))
        np.testing.assert_array_equal(rows, d["hg_%d_rows" % i])
