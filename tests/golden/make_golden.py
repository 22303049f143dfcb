#!/usr/bin/env python3
"""Generate golden input/output vectors by executing the REFERENCE's own numpy-level functions.

TEST INFRASTRUCTURE ONLY — run in the build container, where /root/reference exists:

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What runs: the reference's `FCOS/fcos.py` (`format_data`, `model_loss`, `focal_loss`,
`smooth_l1_loss`, `iou_loss`), `RetinaNet/retinanet_module.py` (`RetinaNet.__init__` anchor dims,
`get_anchors`, `format_data`), `RetinaNet/utils.py:compute_iou`,
`CenterNet/tf_centernet_hourglass.py` (`format_data`, `model_loss`, `nms`, `bboxes_iou`) and
`CenterNet/tf_centernet.py` (`center_dist_1d/2d`, `format_data`), imported from /root/reference with
`tests/golden/tfstub` (numpy stand-ins for TF's elementwise ops, see its docstring) first on
sys.path.  TensorFlow itself is not installed in this image (ordinary ModuleNotFoundError, see
SURVEY.md §8c).  No reference source is copied: only inputs/outputs are written.

Each detector family runs in its own subprocess because FCOS/ and RetinaNet/ both ship modules
named `utils` / `data_preprocess`.
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STUB = os.path.join(HERE, "tfstub")
REF = os.environ.get("CVL_REFERENCE", "/root/reference")


# ----------------------------------------------------------------------------------------------
# synthetic VOC/COCO-shaped boxes (SURVEY.md §8d generator, widened to cover edge cases)
# ----------------------------------------------------------------------------------------------
def synth_boxes(rng, img_h, img_w, n_classes, lam=1.4, nmax=16, side_lo=2.0, side_hi=480.0,
                edge_frac=0.15):
    """Normalised (yc, xc, h, w, cls) float32 rows, distinct areas, optional border-touching."""
    n = int(min(max(1 + rng.poisson(lam), 1), nmax))
    rows, areas = [], set()
    while len(rows) < n:
        h = float(np.exp(rng.uniform(np.log(side_lo), np.log(min(side_hi, img_h)))))
        w = float(np.exp(rng.uniform(np.log(side_lo), np.log(min(side_hi, img_w)))))
        if rng.uniform() < edge_frac:      # touch a border exactly / straddle it slightly
            yc = h / 2.0 if rng.uniform() < 0.5 else img_h - h / 2.0
            xc = rng.uniform(w / 2.0, img_w - w / 2.0)
            if rng.uniform() < 0.3:
                yc -= rng.uniform(0.0, 6.0)
        else:
            yc = rng.uniform(h / 2.0, img_h - h / 2.0)
            xc = rng.uniform(w / 2.0, img_w - w / 2.0)
        r = np.array([yc / img_h, xc / img_w, h / img_h, w / img_w,
                      rng.integers(0, n_classes)], dtype=np.float32)
        a = float(np.float32(r[2] * np.float32(img_h)) * np.float32(r[3] * np.float32(img_w)))
        if a in areas:
            continue
        areas.add(a)
        rows.append(r)
    return np.stack(rows).astype(np.float32)


# ----------------------------------------------------------------------------------------------
# child-process workers (run with the stub + one reference family dir on sys.path)
# ----------------------------------------------------------------------------------------------
def _child_setup(family):
    sys.path.insert(0, os.path.join(REF, family))
    sys.path.insert(0, STUB)
    np.int = int  # reference RetinaNet/retinanet_module.py:303 uses np.int (removed in numpy>=1.24)
    import tensorflow as tf  # the stub
    return tf


def work_fcos(out_path):
    tf = _child_setup("FCOS")
    import fcos as ref
    rng = np.random.default_rng(20250218)
    C = 20
    # (img_dim, img_pad): square bench case, jittered non-square cases padded to x128 squares
    dims = [((512.0, 512.0), (512, 512))] * 24 + [
        ((300.0, 384.0), (384, 384)), ((384.0, 256.0), (384, 384)), ((240.0, 320.0), (384, 384)),
        ((384.0, 384.0), (384, 384)), ((256.0, 256.0), (256, 256)), ((200.0, 256.0), (256, 256)),
        ((128.0, 128.0), (128, 128)), ((333.0, 251.0), (384, 384))] * 4
    assign = {"n_images": len(dims), "C": C}
    arrays = {}
    for i, (dim, pad) in enumerate(dims):
        H, W = dim
        boxes = synth_boxes(rng, H, W, C)
        img_dim = tf.constant(np.array(dim, dtype=np.float32))
        gt = tf.constant(boxes)
        outs, ntgt = ref.format_data(gt, img_dim, C, img_pad=list(pad))
        arrays["assign_%d_boxes" % i] = boxes
        arrays["assign_%d_img_dim" % i] = np.array(dim, dtype=np.float32)
        arrays["assign_%d_img_pad" % i] = np.array(pad, dtype=np.int32)
        arrays["assign_%d_ntgt" % i] = np.array(ntgt, dtype=np.int32)
        for l, o in enumerate(outs):
            arrays["assign_%d_L%d" % (i, l)] = np.asarray(o)
    # losses on reference targets + random logits (fp32), l1 and iou
    loss_imgs = [0, 1, 28, 30, 36, 38, 44, 46]
    assign["loss_imgs"] = loss_imgs
    for i in loss_imgs:
        tgt = [arrays["assign_%d_L%d" % (i, l)] for l in range(5)]
        preds = []
        for l in range(5):
            S = tgt[l].shape
            p = rng.normal(0.0, 1.5, size=(1, S[0], S[1], 5 + C)).astype(np.float32)
            p[..., :4] = np.abs(p[..., :4]) * 3.0
            preds.append(p)
        res = {}
        for reg_type in ("l1", "iou"):
            cls, reg, cen = ref.model_loss(tgt, [tf.constant(p) for p in preds],
                                           [8, 16, 32, 64, 128], reg_type=reg_type, cls_lambda=1.0)
            res[reg_type] = np.array([float(cls), float(reg), float(cen)], dtype=np.float64)
        for l in range(5):
            arrays["loss_%d_pred_L%d" % (i, l)] = preds[l]
        arrays["loss_%d_l1" % i] = res["l1"]
        arrays["loss_%d_iou" % i] = res["iou"]
    # elementwise loss functions on random inputs
    x = rng.normal(0, 3, size=(7, 9, 11)).astype(np.float32)
    y = (rng.uniform(size=(7, 9, 11)) < 0.2).astype(np.float64)
    arrays["focal_x"] = x
    arrays["focal_y"] = y
    arrays["focal_out"] = np.float64(float(ref.focal_loss(y, tf.constant(x))))
    a = rng.normal(0, 1.5, size=(6, 5, 4)).astype(np.float32)
    b = rng.normal(0, 1.5, size=(6, 5, 4)).astype(np.float64)
    m = (rng.uniform(size=(6, 5)) < 0.5).astype(np.float32)
    arrays["sl1_pred"] = a
    arrays["sl1_true"] = b
    arrays["sl1_mask"] = m
    arrays["sl1_out"] = np.float64(float(ref.smooth_l1_loss(b, tf.constant(a),
                                                            mask=tf.constant(m))))
    arrays["sl1_out_nomask"] = np.float64(float(ref.smooth_l1_loss(b, tf.constant(a))))
    # decode helper (fcos.py:112-134)
    xy = np.abs(rng.normal(0, 2, size=(6, 7, 4))).astype(np.float32)
    arrays["p2c_in"] = xy
    arrays["p2c_out"] = np.asarray(ref.prediction_to_corners(tf.constant(xy), 16))
    np.savez_compressed(out_path, meta=json.dumps(assign), **arrays)


def work_retina(out_path):
    tf = _child_setup("RetinaNet")
    import retinanet_module as rm
    import utils as rutils
    rm.build_model = lambda *a, **k: None      # model layers are not part of the golden
    rng = np.random.default_rng(77)
    C = 80
    arrays = {}
    cases = [(640, [20.0, 40.0, 80.0, 160.0, 320.0])] * 3 + \
            [(512, None)] * 2 + [(256, [20.0, 40.0, 80.0, 160.0, 320.0])] * 8 + \
            [(320, [20.0, 40.0, 80.0, 160.0, 320.0])] * 4
    for i, (D, sizes) in enumerate(cases):
        net = rm.RetinaNet(C, {k: str(k) for k in range(C)}, anchor_sizes=sizes)
        dims = np.array([[float(np.asarray(v)) for v in np.asarray(ab, dtype=np.float64)]
                         for lev in net.anchor_boxes for ab in lev], dtype=np.float64)
        boxes = synth_boxes(rng, float(D), float(D), C, lam=6.3, nmax=50, side_lo=8.0,
                            side_hi=float(D), edge_frac=0.1)
        img_dim = tf.constant(np.array([D, D], dtype=np.float32))
        outs, ntgt = net.format_data(tf.constant(boxes), img_dim, iou_thresh=0.5, img_pad=[D, D])
        arrays["case_%d_D" % i] = np.int32(D)
        arrays["case_%d_sizes" % i] = np.array(net.anchor_sizes, dtype=np.float64)
        arrays["case_%d_anchor_dims" % i] = dims.reshape(5, 9, 2)
        arrays["case_%d_boxes" % i] = boxes
        arrays["case_%d_ntgt" % i] = np.int64(ntgt)
        for l in range(5):
            arrays["case_%d_L%d" % (i, l)] = np.stack([np.asarray(o) for o in outs[l]])
        if i == 0:
            anc = net.get_anchors([5, 5], 4)
            arrays["get_anchors_5x5_L4"] = np.stack([np.asarray(a) for a in anc])
    b1 = np.abs(rng.normal(50, 20, size=(7, 4))).astype(np.float32)
    b2 = np.abs(rng.normal(50, 20, size=(13, 4))).astype(np.float32)
    arrays["iou_b1"] = b1
    arrays["iou_b2"] = b2
    arrays["iou_out"] = np.asarray(rutils.compute_iou(b1, b2))
    np.savez_compressed(out_path, **arrays)


def work_centernet(out_path):
    tf = _child_setup("CenterNet")
    import tf_centernet_hourglass as hg
    import tf_centernet as cs
    rng = np.random.default_rng(4242)
    C = 20
    arrays = {}
    for i in range(16):
        D = 512.0 if i < 10 else 384.0
        stride = 4 if i % 2 == 0 else 8
        boxes = synth_boxes(rng, D, D, C, lam=2.4, nmax=20, side_lo=3.0, side_hi=D)
        out, n = hg.format_data(tf.constant(boxes), tf.constant(np.array([D, D], np.float32)), C,
                                img_pad=[int(D), int(D)], stride=stride)
        arrays["hg_%d_boxes" % i] = boxes
        arrays["hg_%d_D" % i] = np.float32(D)
        arrays["hg_%d_stride" % i] = np.int32(stride)
        arrays["hg_%d_out" % i] = np.asarray(out)
        arrays["hg_%d_n" % i] = np.int32(n)
    for i in range(6):
        S = 32 if i < 3 else 16
        y = np.zeros((2, S, S, 4 + C), np.float64)
        y[..., :4] = rng.uniform(0, 3, size=(2, S, S, 4))
        cls_on = rng.uniform(size=(2, S, S)) < 0.05
        y[..., 4:][cls_on, 0] = 1.0
        p = rng.normal(0, 1.5, size=(2, S, S, 4 + C)).astype(np.float32)
        c, r = hg.model_loss(y, tf.constant(p))
        arrays["hgloss_%d_y" % i] = y
        arrays["hgloss_%d_p" % i] = p
        arrays["hgloss_%d_out" % i] = np.array([float(c), float(r)], np.float64)
    for i in range(12):
        D = 512.0 if i < 8 else 384.0
        boxes = synth_boxes(rng, D, D, C, lam=2.4, nmax=20, side_lo=3.0, side_hi=D)
        out = cs.format_data(tf.constant(boxes), tf.constant(np.array([D, D], np.float32)), C,
                             img_pad=[int(D), int(D)], stride=8)
        arrays["splat_%d_boxes" % i] = boxes
        arrays["splat_%d_D" % i] = np.float32(D)
        arrays["splat_%d_out" % i] = np.asarray(out)
    gx = np.arange(3, 9, dtype=np.float64) + 0.5
    gy = np.arange(10, 14, dtype=np.float64) + 0.5
    mx, my = np.meshgrid(gx, gy)
    arrays["cd2_gx"] = mx
    arrays["cd2_gy"] = my
    arrays["cd2_out"] = np.asarray(cs.center_dist_2d(mx, my, mu_x=5, mu_y=12, spread=8.0))
    arrays["cd1_out"] = np.asarray(cs.center_dist_1d(gx, mu_x=6, spread=8.0))
    # nms on random (x, y, w, h, score%, cls) rows: reference nms mutates its input
    for i in range(8):
        n = 40
        xy = rng.uniform(0, 300, size=(n, 2))
        wh = rng.uniform(10, 120, size=(n, 2))
        sc = rng.integers(50, 100, size=(n, 1)).astype(np.float64)
        cl = rng.integers(0, 3, size=(n, 1)).astype(np.float64)
        bb = np.concatenate([xy, wh, sc, cl], axis=1)
        arrays["nms_%d_in" % i] = bb.copy()
        res = hg.nms(bb.copy(), 0.213, method="nms")
        arrays["nms_%d_out" % i] = np.array(res, dtype=np.float64).reshape(-1, 6)
    np.savez_compressed(out_path, **arrays)


def work_retina_decode(out_path):
    """RetinaNet.image_detections / prediction_to_corners / cpu_nms (retinanet_module.py:428-529)
    with the network replaced by fixed synthetic head outputs.  Every row's winning class logit
    is a distinct multiple of 1/1024 and the other classes sit >= 0.5 below it, so scores never
    tie (cpu_nms's quicksort tie order is unspecified) and argmax/threshold decisions sit many
    ulps from any boundary (the sigmoid is ulp-level unpinned)."""
    tf = _child_setup("RetinaNet")
    import retinanet_module as rm
    rm.build_model = lambda *a, **k: None
    rng = np.random.default_rng(91)
    arrays = {}
    cases = [(128, 80, 0.5, 0.05), (256, 20, 0.3, 0.3), (192, 20, 0.5, 0.05), (128, 20, 0.5, 0.9999)]
    for i, (D, C, iou_t, cls_t) in enumerate(cases):
        net = rm.RetinaNet(C, {k: str(k) for k in range(C)}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
        S = [D // s for s in net.strides]
        R = 9 * sum(x * x for x in S)
        win = (rng.permutation(R) - 0.75 * R) / 1024.0
        outs, o = [], 0
        for l in range(5):
            lev = []
            for a in range(9):
                n = S[l] * S[l]
                reg = np.concatenate([rng.normal(0, 0.5, (n, 2)), rng.uniform(0.3, 2.5, (n, 2))], 1)
                cls = win[o:o + n, None] - rng.uniform(0.5, 6.0, (n, C))
                cls[np.arange(n), rng.integers(0, C, n)] = win[o:o + n]
                o += n
                m = np.concatenate([reg, cls], 1).astype(np.float32).reshape(1, S[l], S[l], 4 + C)
                lev.append(m)
            outs.append(lev)
        net.model = lambda x, training=None, _o=outs: [[tf.constant(m) for m in lev] for lev in _o]
        dets = net.image_detections(None, iou_thresh=iou_t, cls_thresh=cls_t)
        arrays["case_%d_cfg" % i] = np.array([D, C, iou_t, cls_t], np.float64)
        arrays["case_%d_anchor_dims" % i] = np.array(net.anchor_boxes, np.float32)
        for l in range(5):
            arrays["case_%d_out_L%d" % (i, l)] = np.concatenate([m for m in outs[l]], 0)
        arrays["case_%d_dets" % i] = np.asarray(dets, np.float32).reshape(-1, 6)
        if i == 0:
            xy = outs[2][4][0][..., :4]
            arrays["corners_in"] = xy
            arrays["corners_dims"] = np.asarray(net.anchor_boxes[2][4], np.float32)
            arrays["corners_out"] = np.asarray(net.prediction_to_corners(xy, net.anchor_boxes[2][4], 32))
            d = np.concatenate([np.sort(rng.uniform(0, 200, (300, 2)), 1)[:, [0, 1]],
                                rng.uniform(0, 200, (300, 2))], 1)
            d = np.stack([d[:, 0], d[:, 2], d[:, 0] + rng.uniform(1, 60, 300), d[:, 2] + rng.uniform(1, 60, 300),
                          rng.permutation(300) / 300.0 + 0.001, np.zeros(300)], 1).astype(np.float32)
            arrays["nms_dets"] = d
            arrays["nms_keep"] = np.asarray(net.cpu_nms(d, 0.45), np.int64)
    np.savez_compressed(out_path, **arrays)


def work_fcos_center(out_path):
    """FCOS/fcos_center.py format_data (train_fcos_center_voc.py: center_only=True; also the 3x3
    default) on synthetic VOC-shaped boxes with distinct areas."""
    tf = _child_setup("FCOS")
    import fcos_center as fc
    rng = np.random.default_rng(123)
    arrays = {}
    C = 20
    for i in range(24):
        D = [512, 384, 640][i % 3]
        boxes = synth_boxes(rng, float(D), float(D), C, lam=2.0 if i < 12 else 30.0, nmax=48, side_lo=4.0,
                            side_hi=float(D) if i < 12 else 60.0, edge_frac=0.2)
        img_dim = np.array([D, D], np.float32)
        co = bool(i % 2)
        outs, nt = fc.format_data(tf.constant(boxes), img_dim, C, img_pad=[D, D], center_only=co)
        arrays["case_%d_boxes" % i] = boxes
        arrays["case_%d_cfg" % i] = np.array([D, int(co)], np.int32)
        arrays["case_%d_ntgt" % i] = np.array(nt, np.int32)
        for l in range(5):
            arrays["case_%d_L%d" % (i, l)] = np.asarray(outs[l]).astype(np.float32)
    np.savez_compressed(out_path, **arrays)


def work_centernet_softnms(out_path):
    """tf_centernet_hourglass.nms(method='soft-nms') (:44-85): the Gaussian-decay branch, on random
    (x, y, w, h, score, cls) rows with distinct scores (ties would be broken by argmax order in
    both; distinct keeps the first-maximum rule out of the float64 exp's last ulp)."""
    tf = _child_setup("CenterNet")
    import tf_centernet_hourglass as hg
    rng = np.random.default_rng(777)
    arrays = {}
    for i in range(8):
        n = [12, 40, 64, 5, 30, 48, 20, 33][i]
        xy = rng.uniform(0, 200, size=(n, 2))
        wh = rng.uniform(10, 120, size=(n, 2))
        sc = (rng.permutation(n) + 1.0).reshape(n, 1) / n * 0.9
        cl = rng.integers(0, 1 + i % 3, size=(n, 1)).astype(np.float64)
        bb = np.concatenate([xy, wh, sc, cl], axis=1)
        sigma = [0.3, 0.5, 0.1, 0.3, 1.0, 0.3, 0.05, 0.3][i]
        arrays["soft_%d_in" % i] = bb.copy()
        arrays["soft_%d_sigma" % i] = np.float64(sigma)
        res = hg.nms(bb.copy(), 0.5, sigma=sigma, method="soft-nms")
        arrays["soft_%d_out" % i] = np.array(res, dtype=np.float64).reshape(-1, 6)
    np.savez_compressed(out_path, **arrays)


def work_fcos_center_v1(out_path):
    """FCOS/fcos_center_v1.py format_data (centroid-cell targets) and model_loss (focal cls + focal
    centerness + smooth-L1 on the sigmoid reg head), plus fcos_center.py's model_loss with
    cen_type="focal" (what train_fcos_center_voc.py trains) on the same random heads."""
    tf = _child_setup("FCOS")
    import fcos_center as fc
    import fcos_center_v1 as f1
    rng = np.random.default_rng(321)
    arrays = {}
    C = 20
    for i in range(16):
        D = [512, 384, 640, 448][i % 4]
        boxes = synth_boxes(rng, float(D), float(D), C, lam=2.0 if i < 8 else 20.0, nmax=40, side_lo=4.0,
                            side_hi=float(D) if i < 8 else 80.0, edge_frac=0.2)
        img_dim = np.array([D, D], np.float32)
        outs, nt = f1.format_data(tf.constant(boxes), img_dim, C, img_pad=[D, D])
        arrays["case_%d_boxes" % i] = boxes
        arrays["case_%d_D" % i] = np.int32(D)
        arrays["case_%d_ntgt" % i] = np.array(nt, np.int32)
        for l in range(5):
            arrays["case_%d_L%d" % (i, l)] = np.asarray(outs[l]).astype(np.float32)
        if i in (1, 5, 9):                  # D = 384: small heads keep the fixture small
            raw = [rng.normal(0, 1.5, size=(1,) + np.asarray(o).shape).astype(np.float32) for o in outs]
            for l in range(5):
                raw[l][..., 4:] -= 2.0
            sig = []
            for r in raw:
                q = r.copy()
                q[..., :4] = np.asarray(tf.nn.sigmoid(tf.constant(r[..., :4])))
                sig.append(tf.constant(q))
            yt = [np.asarray(o, np.float32) for o in outs]
            arrays["loss_%d_out" % i] = np.array([float(v) for v in f1.model_loss(yt, sig)], np.float64)
            arrays["loss_%d_center_focal" % i] = np.array(
                [float(v) for v in fc.model_loss(yt, [tf.constant(r) for r in raw], cen_type="focal")], np.float64)
            for l in range(5):
                arrays["loss_%d_raw_L%d" % (i, l)] = raw[l]
    # prediction_to_corners (:124-147): sigmoid-range offsets/sizes, non-square map
    p = rng.uniform(0.0, 1.0, (12, 9, 5 + C)).astype(np.float32)
    arrays["p2c_in"] = p
    arrays["p2c_out"] = np.asarray(f1.prediction_to_corners(tf.constant(p), 320.0, 16), np.float64)
    np.savez_compressed(out_path, **arrays)


def work_hourglass_v2(out_path):
    """CenterNet v2: the target maps the REFERENCE's own train_hourglass_voc.train() builds
    (:96-160) -- its function definitions are executed (module-level script code is not) with the
    image reader, the augmentation and tf_hourglass_net.train_step replaced by capturing stubs --
    and tf_hourglass_net.model_loss (focal and sigmoid) on random heads."""
    import ast
    import types
    tf = _child_setup("CenterNet")
    import tf_hourglass_net as hg
    path = os.path.join(REF, "CenterNet", "train_hourglass_voc.py")
    tree = ast.parse(open(path).read())
    tree.body = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.Import, ast.ImportFrom))]
    ns = {"__name__": "train_hourglass_voc_defs"}
    exec(compile(tree, path, "exec"), ns)
    captured = []

    def train_step(model, sub_batch_sz, images, bboxes, masks, optimizer, learning_rate=None):
        captured.append((np.asarray(bboxes.numpy(), np.float32), float(learning_rate)))
        return (0.0, 0.0)
    ns["_parse_image"] = lambda f, img_rows, img_cols: np.zeros((img_rows, img_cols, 3), np.float32)
    ns["image_augment"] = lambda img, bbox, p=0.5: (img, bbox)
    ns["tf_obj_detector"] = types.SimpleNamespace(train_step=train_step)
    tf.image = types.SimpleNamespace(pad_to_bounding_box=lambda x, a, b, h, w: np.zeros((h, w, 3), np.float32))
    rng = np.random.default_rng(777)
    C, n_data, batch, steps = 20, 40, 4, 6
    data = []
    for i in range(n_data):
        n = int(rng.integers(1, 25 if i % 3 else 60))
        cen = rng.uniform(0.02, 0.98, (n, 2))
        if i % 5 == 0:                       # clustered centres: shared cells / scales
            cen = 0.5 + rng.normal(0, 0.02, (n, 2))
        side = np.exp(rng.uniform(np.log(0.01), np.log(1.0), (n, 2)))
        lo, hi = cen - side / 2, cen + side / 2
        bbox = np.concatenate([lo, hi], 1).astype(np.float32)
        if i % 7 == 3:
            bbox[0, [0, 2]] = bbox[0, [2, 0]]   # negative width: skipped by the builder
        data.append({"image": "img_%d.jpg" % i, "objects": {"bbox": bbox,
                                                            "label": rng.integers(0, C, n).astype(np.int64)}})
    ckpt = types.SimpleNamespace(step=types.SimpleNamespace(assign_add=lambda v: None))
    np.random.seed(4321)
    ns["train"](None, C, 2, batch, data, [], 0, steps, None, ckpt, None, {}, init_lr=1e-3, min_lr=1e-5,
                decay=0.99, display_step=10 ** 9, step_cool=10 ** 9)
    np.random.seed(4321)
    arrays = {"C": np.int32(C)}
    for st in range(steps):
        sample = np.random.choice(n_data, size=batch, replace=False)
        rnd = np.random.uniform(low=0.6, high=1.3)
        bbox, lr = captured[st]
        raw = int(rnd * 320)
        img = bbox.shape[1] * 8
        arrays["step_%d_raw_img" % st] = np.array([raw, img], np.int32)
        arrays["step_%d_lr" % st] = np.float64(lr)
        nmax = max(len(data[k]["objects"]["label"]) for k in sample)
        boxes = np.zeros((batch, nmax, 5), np.float32)
        nbox = np.zeros(batch, np.int32)
        for j, k in enumerate(sample):
            o = data[k]["objects"]
            boxes[j, :len(o["label"]), :4] = o["bbox"]
            boxes[j, :len(o["label"]), 4] = o["label"]
            nbox[j] = len(o["label"])
        arrays["step_%d_boxes" % st] = boxes
        arrays["step_%d_nbox" % st] = nbox
        arrays["step_%d_targets" % st] = bbox
    # model_loss on random heads of two captured batches
    for st in (0, 3):                       # 2 images, a 16x16 window around the map centre
        S = arrays["step_%d_targets" % st].shape[1]
        bbox = np.ascontiguousarray(arrays["step_%d_targets" % st][:2, S // 2 - 8:S // 2 + 8, S // 2 - 8:S // 2 + 8])
        arrays["loss_%d_targets" % st] = bbox
        raw = rng.normal(0.0, 1.5, bbox.shape).astype(np.float32)
        bfocal = np.float32(np.log((1.0 - 0.99) / 0.99))
        outs = np.concatenate([np.asarray(tf.nn.sigmoid(tf.constant(raw[..., :4])).numpy(), np.float32),
                               raw[..., 4:] + bfocal], -1)
        arrays["loss_%d_raw" % st] = raw
        arrays["loss_%d_bfocal" % st] = np.float32(bfocal)
        for lt in ("focal", "sigmoid"):
            cls_l, reg_l = hg.model_loss(tf.constant(bbox), tf.constant(bbox[..., 4]), tf.constant(outs),
                                         loss_type=lt)
            arrays["loss_%d_%s" % (st, lt)] = np.array([float(cls_l), float(reg_l)], np.float64)
    np.savez_compressed(out_path, **arrays)


def work_centernet_s8(out_path):
    """CenterNet/tf_centernet_resnet_s8.py format_data (fed as train_centernet_crowdhuman.py does: a
    float32 box array concatenated with the int64 class column -> float64 rows, img_dim the resized
    [raw, raw], img_pad [img, img]) and model_loss on random heads."""
    tf = _child_setup("CenterNet")
    import tf_centernet_resnet_s8 as s8
    rng = np.random.default_rng(808)
    arrays = {}
    scales = [32.0, 64.0, 128.0, 256.0, 512.0]
    C = 3
    for i in range(12):
        img = [512, 384, 256][i % 3]
        raw = img - int(rng.integers(0, 96)) if i % 4 else img
        n = int(rng.integers(1, 40))
        y = rng.uniform(0.02, 0.98, n)
        x = rng.uniform(0.02, 0.98, n)
        h = np.exp(rng.uniform(np.log(0.01), np.log(0.99), n))
        w = np.exp(rng.uniform(np.log(0.01), np.log(0.99), n))
        if i % 5 == 1:                           # crowded: shared cells / scales
            y = 0.5 + rng.normal(0, 0.01, n)
            x = 0.5 + rng.normal(0, 0.01, n)
        box = np.stack([y, x, h, w], 1).astype(np.float32)
        cls = rng.integers(0, C, n).astype(np.int64)[:, None]
        rows = np.concatenate((box, cls), axis=1)          # float64, as the trainer's gt_labels
        out, nt = s8.format_data(tf.constant(rows), scales, [raw, raw], C, img_pad=[img, img], stride=8)
        arrays["case_%d_rows" % i] = np.concatenate([box, cls.astype(np.float32)], 1)
        arrays["case_%d_dims" % i] = np.array([raw, img], np.int32)
        arrays["case_%d_out" % i] = np.asarray(out).astype(np.float32)
        arrays["case_%d_n" % i] = np.int32(nt)
    # model_loss on a 2-image batch (targets of cases 2 and 5: 256 / 384 -> crop both to 32x32)
    yt = np.stack([arrays["case_2_out"][:32, :32], arrays["case_5_out"][:32, :32]])
    rl = rng.normal(0, 1.5, yt.shape[:-1] + (4,)).astype(np.float32)
    cl = rng.normal(-1.0, 2.0, yt.shape[:-1] + (C,)).astype(np.float32)
    pred = np.concatenate([np.asarray(tf.nn.sigmoid(tf.constant(rl)).numpy(), np.float32), cl], -1)
    lc, lr = s8.model_loss(tf.constant(yt), tf.constant(pred))
    arrays["loss_y"], arrays["loss_reg_logits"], arrays["loss_cls_logits"] = yt, rl, cl
    arrays["loss_out"] = np.array([float(lc), float(lr)], np.float64)
    np.savez_compressed(out_path, **arrays)


WORKERS = {"fcos": work_fcos, "retinanet": work_retina, "centernet": work_centernet,
           "fcos_center_v1": work_fcos_center_v1, "hourglass_v2": work_hourglass_v2, "centernet_s8": work_centernet_s8,
           "centernet_softnms": work_centernet_softnms,
           "retina_decode": work_retina_decode,
           "fcos_center": work_fcos_center}


def work_loss_kwargs(out_path):
    """FCOS/fcos.py focal_loss / smooth_l1_loss and RetinaNet/retinanet_module.py's methods of the same
    names at NON-default keyword values (alpha, gamma, delta) and with soft (non-binary) float
    masks / labels: the keyword surface of the drop-in loss functions."""
    tf = _child_setup("FCOS")
    import fcos as ref
    rng = np.random.default_rng(4242)
    arrays, meta = {}, {"focal": [], "sl1": []}
    for k, (alpha, gamma, soft) in enumerate([(0.25, 2.0, False), (0.5, 1.0, False), (0.1, 3.0, True),
                                              (0.75, 0.0, True), (0.25, 1.5, True), (0.9, 2.5, False)]):
        x = rng.normal(0, 3, size=(9, 7, 13)).astype(np.float32)
        y = rng.uniform(size=(9, 7, 13)) if soft else (rng.uniform(size=(9, 7, 13)) < 0.2).astype(np.float64)
        arrays["focal_%d_x" % k] = x
        arrays["focal_%d_y" % k] = y.astype(np.float32)
        arrays["focal_%d_out" % k] = np.float64(float(ref.focal_loss(y.astype(np.float32), tf.constant(x),
                                                                     alpha=alpha, gamma=gamma)))
        meta["focal"].append([alpha, gamma])
    for k, (delta, mask_kind) in enumerate([(1.0, "soft"), (0.5, "binary"), (2.0, "soft"), (0.25, "none"),
                                            (3.0, "binary")]):
        a = rng.normal(0, 1.5, size=(8, 6, 4)).astype(np.float32)
        b = rng.normal(0, 1.5, size=(8, 6, 4)).astype(np.float32)
        arrays["sl1_%d_pred" % k] = a
        arrays["sl1_%d_true" % k] = b
        if mask_kind == "none":
            out = ref.smooth_l1_loss(b, tf.constant(a), delta=delta)
        else:
            m = (rng.uniform(size=(8, 6)) if mask_kind == "soft"
                 else (rng.uniform(size=(8, 6)) < 0.5)).astype(np.float32)
            arrays["sl1_%d_mask" % k] = m
            out = ref.smooth_l1_loss(b, tf.constant(a), mask=tf.constant(m), delta=delta)
        arrays["sl1_%d_out" % k] = np.float64(float(out))
        meta["sl1"].append([delta, mask_kind])
    np.savez_compressed(out_path, meta=json.dumps(meta), **arrays)


WORKERS["loss_kwargs"] = work_loss_kwargs


def work_image_augment(out_path):
    """CenterNet v2 `image_augment` (train_hourglass_voc.py:24-67): the REFERENCE's own function (its
    definition executed from the file; module-level code is not) on random padded images and
    float64 target maps.  The TF image ops it calls are given here: tf.transpose; random_brightness
    = x + delta and random_contrast = (x - mean) * f + mean (per-channel mean over the pixels), the
    magnitudes drawn from a recorded second generator.  Per case: the numpy seed set before the
    call (its np.random.uniform() draws pick the branch), the second generator's seed, inputs and
    outputs."""
    import ast
    import types
    tf = _child_setup("CenterNet")
    path = os.path.join(REF, "CenterNet", "train_hourglass_voc.py")
    tree = ast.parse(open(path).read())
    tree.body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "image_augment"]
    ns = {"np": np, "tf": tf}
    exec(compile(tree, path, "exec"), ns)
    state = {}

    def random_brightness(img, max_delta):
        d = np.float32(state["tf_rng"].uniform(-max_delta, max_delta))
        return tf.Tensor((np.asarray(img.numpy(), np.float32) + d).astype(np.float32))

    def random_contrast(img, lower, upper):
        f = np.float32(state["tf_rng"].uniform(lower, upper))
        a = np.asarray(img.numpy(), np.float32)
        m = a.astype(np.float64).mean(axis=(0, 1)).astype(np.float32)
        return tf.Tensor(((a - m) * f + m).astype(np.float32))
    tf.image = types.SimpleNamespace(random_brightness=random_brightness, random_contrast=random_contrast)
    tf.transpose = lambda x, perm: tf.Tensor(np.transpose(x.numpy() if isinstance(x, tf.Tensor) else x, perm))
    rng = np.random.default_rng(2402)
    C = 3
    arrays = {}
    k = 0
    for N in [20] * 18 + [36] * 6:
        S = (N + 7) // 8
        img = np.zeros((N, N, 3), np.float32)
        pad = int(rng.integers(0, 4))
        img[pad:N - pad, pad:N - pad] = rng.uniform(0, 1, (N - 2 * pad, N - 2 * pad, 3)).astype(np.float32)
        bbox = np.zeros((S, S, 4, 5 + C))
        for _ in range(int(rng.integers(1, 6))):
            y, x, sc = int(rng.integers(0, S)), int(rng.integers(0, S)), int(rng.integers(0, 4))
            bbox[y, x, sc, :4] = [rng.uniform(), rng.uniform(), rng.uniform(0.1, 2), rng.uniform(0.1, 2)]
            bbox[y, x, sc, 4] = 1.0
            bbox[y, x, sc, 5 + int(rng.integers(0, C))] = 1.0
        seed_np, seed_tf = 1000 + k, 5000 + k
        state["tf_rng"] = np.random.RandomState(seed_tf)
        np.random.seed(seed_np)
        out_img, out_bbox = ns["image_augment"](tf.constant(img), bbox.copy())
        arrays["case_%d_seeds" % k] = np.array([seed_np, seed_tf], np.int64)
        arrays["case_%d_img" % k] = img
        arrays["case_%d_bbox" % k] = bbox
        arrays["case_%d_out_img" % k] = np.asarray(out_img.numpy() if hasattr(out_img, "numpy") else out_img,
                                                   np.float32)
        arrays["case_%d_out_bbox" % k] = np.asarray(out_bbox.numpy() if hasattr(out_bbox, "numpy") else out_bbox,
                                                    np.float64)
        k += 1
    arrays["n_cases"] = np.int32(k)
    np.savez_compressed(out_path, **arrays)


WORKERS["image_augment"] = work_image_augment


def work_variant_decode(out_path):
    """The numeric part of the variant CenterNets' `obj_detect_results`: the REFERENCE's own functions
    (CenterNet/tf_centernet_resnet_s8.py:446-600 with its prediction_to_corners and nms;
    CenterNet/tf_hourglass_net.py:451-600), called with a model whose predict() returns a fixed
    random head, the image reader / PIL / matplotlib replaced by recording stand-ins (heatmap=False).
    Recorded per case: the head, the call's arguments, the rows the s8 function hands to `nms` and
    what `nms` returns, and the v2 function's drawn rectangles + texts as (x_lower, y_lower,
    box_width, box_height, prob %, label index) rows.  tf.nn.sigmoid is evaluated in float64 and
    rounded to fp32 (TF's fp32 kernel is not available: its last ulp is unpinned either way)."""
    import types
    tf = _child_setup("CenterNet")
    tf.nn.sigmoid = staticmethod(lambda x: tf.Tensor(
        (1.0 / (1.0 + np.exp(-np.asarray(x.numpy() if isinstance(x, tf.Tensor) else x, np.float64))))
        .astype(np.float32)))
    import tf_centernet_resnet_s8 as s8
    import tf_hourglass_net as hg
    state = {}

    class _Ax(object):
        def imshow(self, *a, **k):
            return None

        def add_patch(self, p):
            state["rects"].append(p)

        def text(self, x, y, t, **k):
            state["texts"].append((x, y, t))

    class _Fig(object):
        def colorbar(self, *a, **k):
            pass

        def suptitle(self, *a, **k):
            pass

        def savefig(self, *a, **k):
            pass
    plt = types.SimpleNamespace(subplots=lambda n: (_Fig(), _Ax()), close=lambda: None,
                                Rectangle=lambda xy, w, h, **k: (float(xy[0]), float(xy[1]), float(w), float(h)))
    image = types.SimpleNamespace(open=lambda f: np.zeros(state["img_shape"] + (3,), np.uint8))
    ref_nms = s8.nms

    def nms_rec(bboxes, iou_threshold, sigma=0.3, method="nms"):
        state["nms_in"] = np.array(bboxes, np.float64).copy()
        out = ref_nms(bboxes, iou_threshold, sigma, method)
        state["nms_out"] = np.array(out, np.float64).reshape(-1, 6)
        return out
    for mod in (s8, hg):
        mod.plt = plt
        mod.Image = image
        mod._parse_image = lambda f, img_rows=448, img_cols=448: np.zeros((img_rows, img_cols, 3), np.float32)
    s8.nms = nms_rec

    class _Model(object):
        def predict(self, x):
            return state["head"][None]
    rng = np.random.default_rng(4471)
    arrays = {}
    # s8: (S, n_scales, C, thresh, downsample, img rows/cols, source image shape)
    s8_cases = [(24, 5, 3, 0.5, 8, (192, 192), (375, 500)), (28, 3, 1, 0.4, 8, (224, 224), (224, 224)),
                (16, 5, 6, 0.6, 8, (128, 128), (640, 427)), (20, 2, 2, 0.99, 8, (160, 160), (160, 160))]
    for i, (S, ns, C, thr, ds, (ir, ic), shp) in enumerate(s8_cases):
        head = np.zeros((S, S, ns, 4 + C), np.float32)
        head[..., :2] = rng.uniform(-0.3, 1.3, (S, S, ns, 2))
        head[..., 2:4] = rng.uniform(0.0, 1.2, (S, S, ns, 2))
        head[..., 4:] = rng.normal(-3.5, 2.0, (S, S, ns, C))
        scales = [16.0, 32.0, 64.0, 128.0, 256.0][:ns]
        state.update(head=head, img_shape=shp, rects=[], texts=[], nms_in=np.zeros((0, 6)), nms_out=np.zeros((0, 6)))
        s8.obj_detect_results("img.jpg", _Model(), scales, ["c%d" % k for k in range(C)], heatmap=False, thresh=thr,
                              downsample=ds, iou_thresh=0.213, img_rows=ir, img_cols=ic)
        arrays["s8_%d_head" % i] = head
        arrays["s8_%d_args" % i] = np.array([thr, ds, ir, ic, shp[0], shp[1]], np.float64)
        arrays["s8_%d_scales" % i] = np.array(scales, np.float64)
        arrays["s8_%d_raw" % i] = state["nms_in"]
        arrays["s8_%d_nms" % i] = state["nms_out"]
    # v2: (S, C classes incl. channel 0, thresh, img rows/cols, img_scale, source image shape)
    hg_cases = [(24, 4, 0.5, (192, 192), None, (375, 500)), (28, 1, 0.45, (224, 224), None, (224, 224)),
                (16, 6, 0.6, (128, 128), [32, 64, 96, 100], (640, 427)), (40, 3, 0.55, (320, 320), None, (512, 512))]
    for i, (S, C, thr, (ir, ic), isc, shp) in enumerate(hg_cases):
        head = np.zeros((S, S, 4, 4 + C), np.float32)
        head[..., :2] = rng.uniform(-0.2, 1.2, (S, S, 4, 2))
        head[..., 2:4] = rng.uniform(0.0, 3.0, (S, S, 4, 2))
        head[..., 4:] = rng.normal(-3.5, 2.0, (S, S, 4, C))
        state.update(head=head, img_shape=shp, rects=[], texts=[])
        labels = ["c%d" % k for k in range(C)]
        hg.obj_detect_results("img.jpg", _Model(), labels, heatmap=False, thresh=thr, img_rows=ir, img_cols=ic,
                              img_scale=isc)
        rows = []
        for (y_lo, x_lo, bh, bw), (_, _, t) in zip(state["rects"], state["texts"]):
            lab, pr = t.split(": ")
            rows.append([x_lo, y_lo, bw, bh, float(pr.rstrip("%")), float(labels.index(lab))])
        arrays["hg_%d_head" % i] = head
        arrays["hg_%d_args" % i] = np.array([thr, ir, ic, shp[0], shp[1]], np.float64)
        arrays["hg_%d_scale" % i] = np.array(isc if isc is not None else [], np.float64)
        arrays["hg_%d_rows" % i] = np.array(rows, np.float64).reshape(-1, 6)
    arrays["n_s8"], arrays["n_hg"] = np.int32(len(s8_cases)), np.int32(len(hg_cases))
    np.savez_compressed(out_path, **arrays)


WORKERS["variant_decode"] = work_variant_decode


def main():
    if len(sys.argv) == 3 and sys.argv[1] in WORKERS:
        WORKERS[sys.argv[1]](sys.argv[2])
        return
    if not os.path.isdir(REF):
        print("reference not present at %s: nothing to do" % REF)
        return
    only = sys.argv[1:]                   # optional: regenerate only these families
    for fam in WORKERS:
        if only and fam not in only:
            continue
        out = os.path.join(HERE, "golden_%s.npz" % fam)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), fam, out])
        print("wrote", out, os.path.getsize(out), "bytes")
    with open(os.path.join(HERE, "GOLDEN_INFO.json"), "w") as f:
        json.dump({"numpy": np.__version__, "python": sys.version.split()[0],
                   "generator": "tests/golden/make_golden.py",
                   "reference": "WD-Leong/CV-Lite-Object-Detection @ 2025-02-18"}, f, indent=1)


if __name__ == "__main__":
    main()
