"""Host-side logic of the cvlite mirrors that runs without a GPU: anchor dimensions (RetinaNet
__init__, retinanet_module.py:205-219) and the resize/pad plan of resize_and_pad_image
(data_preprocess.py:41-96), checked against the oracle restatements / reference goldens."""
import numpy as np
import pytest

from oracle import preprocess_ref, retina_ref


def test_retina_anchor_dims_host_match_goldens(golden):
    from cvlite.retinanet import RetinaNet
    d = golden("retinanet")
    i = 0
    while "case_%d_D" % i in d:
        net = RetinaNet(80, {}, anchor_sizes=list(d["case_%d_sizes" % i]))
        np.testing.assert_array_equal(np.array(net.anchor_boxes, np.float64), d["case_%d_anchor_dims" % i])
        np.testing.assert_array_equal(np.array(net.anchor_boxes, np.float32),
                                      retina_ref.anchor_dims(list(d["case_%d_sizes" % i])))
        i += 1
    assert i > 0
    with pytest.raises(ValueError):
        RetinaNet(80, {}, anchor_sizes=[1.0, 2.0])


@pytest.mark.parametrize("H,W,mn,mx,stride,eq", [
    (375, 500, 512.0, 512.0, 128.0, True), (500, 333, 800.0, 1333.0, 128.0, True),
    (480, 640, 600.0, 1000.0, 32.0, False), (1024, 768, 417.3, 600.0, 128.0, True)])
def test_resize_plan_matches_restatement(H, W, mn, mx, stride, eq):
    from cvlite.data_preprocess import _plan
    new_shape, ratio, ph, pw = _plan(H, W, None, mn, mx, stride, eq, None)
    img, rns, rratio = preprocess_ref.resize_and_pad_image(np.zeros((H, W, 3), np.uint8), mn, mx, stride, eq)
    np.testing.assert_array_equal(new_shape, rns)
    assert ratio == rratio and (ph, pw) == img.shape[:2]


def test_checkpoint_manager_roundtrip_cpu(tmp_path):
    """tf.train.Checkpoint / CheckpointManager mirror (cvlite.checkpoint): numbered saves,
    max_to_keep pruning, latest_checkpoint, step counter, parameters + momentum + BN moving
    statistics restored, layout mismatch rejected.  CPU tensors stand in for the device store."""
    import torch
    from cvlite import checkpoint as ck
    from cvlite.layers import BatchNorm, ParamStore, constant

    class Net(object):
        def __init__(self, seed, extra=False):
            self.store = ParamStore()
            self.store.add("a/kernel", (3, 4), constant(seed))
            self.bn = BatchNorm(self.store, "a_bn", 4)
            if extra:
                self.store.add("b/kernel", (2,), constant(0.0))
            self.store.finalize("cpu", int(seed))
            self.bn.init_buffers("cpu")
            self.packed = 0

        def bns(self):
            return [self.bn]

        def pack(self):
            self.packed += 1

    net = Net(1.0)
    net.store.mom.fill_(0.5)
    net.bn.run_mean.fill_(0.25)
    c = ck.Checkpoint(step=ck.Variable(0), model=net)
    m = ck.CheckpointManager(c, str(tmp_path), max_to_keep=2)
    assert m.latest_checkpoint is None
    for i in range(3):
        c.step.assign_add(1)
        m.save()
    assert [p.rsplit("-", 1)[1] for p in m.checkpoints] == ["2.pt", "3.pt"]
    assert m.latest_checkpoint.endswith("ckpt-3.pt")
    other = Net(2.0)
    c2 = ck.Checkpoint(step=ck.Variable(0), model=other)
    c2.restore(m.latest_checkpoint)
    assert int(c2.step.numpy()) == 3 and other.packed == 1
    assert torch.equal(other.store.flat, net.store.flat) and torch.equal(other.store.mom, net.store.mom)
    assert torch.equal(other.bn.run_mean, net.bn.run_mean)
    # a manager re-opened on the same directory continues the numbering
    assert ck.CheckpointManager(c, str(tmp_path), max_to_keep=2).save().endswith("ckpt-4.pt")
    with pytest.raises(ValueError):
        ck.Checkpoint(model=Net(3.0, extra=True)).restore(m.latest_checkpoint)


def test_preprocess_box_path_and_size_plan():
    """preprocess_data's box path (FCOS/data_preprocess.py:120-131: random_flip_horizontal's box map,
    utils.swap_xy, utils.convert_to_xywh) and the host size plan used to bucket jittered batches:
    square padded sizes, multiples of 128, new_shape = ratio * shape in fp32."""
    import numpy as np
    from cvlite.data_preprocess import box_targets, padded_size
    b = np.array([[0.1, 0.2, 0.5, 0.9], [0.0, 0.3, 1.0, 0.4]], np.float32)
    for flip in (False, True):
        t = b.copy()
        if flip:
            t = np.stack([1 - b[:, 2], b[:, 1], 1 - b[:, 0], b[:, 3]], -1).astype(np.float32)
        s = t[:, [1, 0, 3, 2]]
        exp = np.concatenate([(s[:, :2] + s[:, 2:]) / np.float32(2), s[:, 2:] - s[:, :2]], -1)
        np.testing.assert_array_equal(box_targets(b, flip), exp)
    rng = np.random.default_rng(0)
    for _ in range(20):
        flip, shp, S = padded_size((375, 500), [640, 1024], 800.0, 1333.0, rng)
        assert S % 128 == 0 and S >= shp.max() and shp.dtype == np.float32
        assert 640 - 1e-3 <= shp.min() <= 1024 + 1e-3 or shp.max() <= 1333.0 + 1e-3


def test_parse_image_decodes_files(tmp_path):
    """_parse_image (FCOS/data_preprocess.py:5-9) reads a JPEG / PNG file into [H,W,3] uint8 (PNG:
    lossless, so the decode must return the written pixels exactly)."""
    import numpy as np
    from PIL import Image
    from cvlite.data_preprocess import _parse_image
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (37, 53, 3)).astype(np.uint8)
    Image.fromarray(a).save(tmp_path / "x.png")
    np.testing.assert_array_equal(_parse_image(str(tmp_path / "x.png")), a)
    yy, xx = np.mgrid[0:37, 0:53]
    sm = np.stack([yy * 6, xx * 4, (yy + xx) * 2], -1).astype(np.uint8)     # smooth: JPEG-friendly
    Image.fromarray(sm).save(tmp_path / "x.jpg", quality=95)
    j = _parse_image(str(tmp_path / "x.jpg"))
    assert j.shape == (37, 53, 3) and j.dtype == np.uint8 and np.abs(j.astype(int) - sm).mean() < 3


def test_fcos_center_resnet101_branch():
    """fcos_center.py:37-43 / fcos_center_v1.py:37-43 build ResNet-101 for "resnet101"; fcos.py:
    29-41 has no such branch (every non-resnet50 name is MobileNetV2)."""
    from cvlite.fcos_center_net import FCOSCenterNet
    from cvlite.fcos_net import FCOSNet
    p = FCOSCenterNet.param_dict(20, backbone_model="resnet101")
    assert "conv4_block23_3_conv/kernel" in p and "conv4_block24_1_conv/kernel" not in p
    assert "cen_output_1/kernel" in p
    assert "Conv1/kernel" in FCOSNet.param_dict(20, backbone_model="resnet101")
    assert "conv4_block6_3_conv/kernel" in FCOSCenterNet.param_dict(20, backbone_model="resnet50")
    assert "Conv1/kernel" in FCOSCenterNet.param_dict(20, backbone_model="mobilenetv2")


def test_parse_image_decodes_jpeg_and_png(tmp_path):
    """data_preprocess._parse_image (FCOS/data_preprocess.py:5-9): a JPEG / PNG file -> [H,W,3] uint8
    (host PIL decode, RGB; grayscale and RGBA inputs are converted like decode_jpeg(channels=3))."""
    import numpy as np
    from PIL import Image
    from cvlite.data_preprocess import _parse_image
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    p = str(tmp_path / "a.png")
    Image.fromarray(img).save(p)
    np.testing.assert_array_equal(_parse_image(p), img)                 # lossless
    q = str(tmp_path / "a.jpg")
    Image.fromarray(img).save(q, quality=95)
    with Image.open(q) as im:
        ref = np.asarray(im.convert("RGB"))
    np.testing.assert_array_equal(_parse_image(q), ref)
    g = str(tmp_path / "g.jpg")
    Image.fromarray(img[..., 0]).save(g)
    assert _parse_image(g).shape == (37, 53, 3)


def test_bn_acc_encoding_exact_and_order_independent():
    """BN accumulators (include/cvlite.h, csrc/bn_acc.h): the host encoder equals a plain-Python
    restatement of the bin split; partials added in any order give identical bins; the decoded value
    is exact for |x| in [2^-40, 2^54)."""
    import math
    import struct

    import torch
    from cvlite import ops_nn as nn

    def split(p):
        u = struct.unpack("<I", struct.pack("<f", p))[0]
        e = (u >> 23) & 0xFF
        if e == 255:
            return 7, 1
        r = e - 27
        if e == 0 or r < 0:
            return None, 0
        k = r // 22
        if k >= 7:
            return 7, 1
        m = ((u & 0x7FFFFF) | 0x800000) << (r - 22 * k)
        return k, (-m if u >> 31 else m)

    def encode(x):
        bins = [0] * 8
        hi = float(np.float32(x))
        r = x - hi
        mid = float(np.float32(r))
        for p in (hi, mid, float(np.float32(r - mid))):
            k, v = split(p)
            if k is not None:
                bins[k] += v
        return bins

    def decode(b):
        if b[7]:
            return float("nan")
        t = 0.0
        for k in range(7):
            t += float(b[k]) * math.ldexp(1.0, 27 + 22 * k - 150)
        return t

    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.standard_normal(300) * 10.0 ** rng.integers(-12, 15, 300),
                           [0.0, -0.0, 1e-40, 2.0 ** 60, float("inf"), float("nan")]])
    acc = nn.bn_acc_encode(torch.tensor(vals).view(-1, 1).repeat(1, 2), exact=True)
    for i, x in enumerate(vals):
        b = encode(float(x))
        assert acc[i, 0].tolist() == b, (x, acc[i, 0].tolist(), b)
        if np.isfinite(x) and 2.0 ** -40 <= abs(x) < 2.0 ** 54:
            assert decode(b) == x
    # fp32 partials summed in two orders: the bins (integers) agree exactly
    parts = (rng.standard_normal(4096) * 10.0 ** rng.integers(-6, 6, 4096)).astype(np.float32)
    b1, b2 = [0] * 8, [0] * 8
    for p in parts:
        k, v = split(float(p))
        b1[k] += v
    for p in parts[::-1][rng.permutation(len(parts))]:
        k, v = split(float(p))
        b2[k] += v
    assert b1 == b2
    exact = math.fsum(float(p) for p in parts)
    assert abs(decode(b1) - exact) <= 1e-15 * abs(exact) + 1e-300
