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
