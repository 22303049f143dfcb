"""Keras-name weight interchange (cvlite.checkpoint): export -> import into a
differently initialised network reproduces every parameter, BN statistic and the inference
outputs bit-exactly; RetinaNet's fused heads are split into the reference's per-(level, anchor)
Keras variables (retinanet_module.py:115-148) with the reference's shapes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _roundtrip(make, tmp_path, H, n_reg, n_cls):
    from cvlite import checkpoint
    a, b = make(0), make(1)
    for bn in checkpoint._bns(a):                  # non-trivial running statistics
        bn.run_mean.uniform_(-1, 1)
        bn.run_var.uniform_(0.5, 2)
    p = str(tmp_path / "w.npz")
    checkpoint.export_keras_weights(a, p)
    assert not torch.equal(a.store.flat, b.store.flat)
    checkpoint.import_keras_weights(b, p)
    assert torch.equal(a.store.flat, b.store.flat)
    for x, y in zip(checkpoint._bns(a), checkpoint._bns(b)):
        assert torch.equal(x.run_mean, y.run_mean) and torch.equal(x.run_var, y.run_var)
    img = torch.rand((1, H, H, 3), device="cuda") * 2 - 1
    ra, ca = a.forward(img, train=False)
    rb, cb = b.forward(img, train=False)
    # padding channels past the heads' outputs are never written: compare the stored ones
    assert torch.equal(ra[..., :n_reg], rb[..., :n_reg]) and torch.equal(ca[..., :n_cls], cb[..., :n_cls])
    return np.load(p, allow_pickle=False)


def test_fcos_keras_weights_roundtrip(tmp_path):
    from cvlite.fcos_net import FCOSNet
    z = _roundtrip(lambda s: FCOSNet(20, device=torch.device("cuda", 0), seed=s), tmp_path, 128, 5, 20)
    assert z["conv2_block1_1_conv/kernel:0"].shape == (1, 1, 64, 64)
    assert z["conv5_block3_3_bn/moving_variance:0"].shape == (2048,)
    assert z["logits_output_1/kernel:0"].shape[-1] == 20


def test_retinanet_keras_weights_per_anchor(tmp_path):
    from cvlite import checkpoint
    from cvlite.retina_net import RetinaNetNet
    z = _roundtrip(lambda s: RetinaNetNet(80, device=torch.device("cuda", 0), seed=s), tmp_path, 128,
                   36, 720)
    for l in range(1, 6):
        for a in range(1, 10):
            assert z["cls_output_%d_anchor_%d/kernel:0" % (l, a)].shape == (3, 3, 256, 80)
            assert z["reg_output_%d_anchor_%d/bias:0" % (l, a)].shape == (4,)
    with pytest.raises(KeyError):
        w = {k: z[k] for k in z.files if k != "cls_output_3_anchor_7/bias:0"}
        checkpoint.load_keras_weights(RetinaNetNet(80, device=torch.device("cuda", 0), seed=2), w)
