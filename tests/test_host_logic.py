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
