"""BASELINE.json configs[0] on the HIP path: `FCOS/train_fcos.py:87-251 train` on 8 synthetic VOC
512x512 images, batch_size 8, one step -- called through the drop-in loop
`cvlite.train_fcos.train(...)` with the reference's keyword surface and pre-processed samples
(dict(image [512,512,3] in [-1, 1], bbox [N,4] normalised (yc, xc, h, w), label [N])).

* fp32 parity mode (CVL_PRECISION=fp32): the loop's one update vs
  oracle/model_ref.train_step_reference (the reference's per-image batch-1 gradient sum, /bs,
  clip_by_global_norm(1.0), Keras SGD momentum 0.9; train_fcos.py:128-185) run in float64 on the
  same images (in the loop's own np.random order, train_fcos.py:112), targets and initial
  weights.  Residual-branch BN gammas damped x0.25 (the well-conditioned graph of
  test_gpu_parity_fp32.py).  Tolerances: per-image losses rel 1e-4; momentum (= -lr x the clipped
  mean gradient after one step) flat rel-L2 <= max(1e-4, 1.5 x the fp32 oracle's own distance
  from float64: ReLU-mask noise, test_gpu_parity_fp32.py docstring); parameters rel-L2 1e-4.
* production bf16: the same loop run eagerly (the kernels the HIP graphs capture) inside
  tests/launch_parity.py's LaunchParity -- every launch of the step teacher-forced against float64
  torch on the GPU's own inputs (bf16 rel-L2 1e-2, fp32 1e-4) and every C entry point checked --
  plus the per-image losses the fused loss kernel reported vs the oracle loss
  (oracle/fcos_ref.model_loss, pinned to the reference's fcos.model_loss by the goldens) on the
  GPU's own head outputs: rtol 2e-5; targets bit-exact vs fcos_ref.format_data."""
import math

import numpy as np
import pytest
import torch

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu

C, B, S, SEED = 20, 8, 512, 31
LOSS_RTOL_F32 = 1e-4
MOM_RTOL = 1e-4
NOISE_X = 1.5


def _samples():
    from cvlite.train_fcos import synthetic_batch
    imgs, boxes, nbox = synthetic_batch(B, S, S, C, seed=2026, device="cpu")
    out = []
    for b in range(B):
        n = int(nbox[b])
        out.append(dict(image=imgs[b].numpy(), bbox=boxes[b, :n, :4].numpy().copy(),
                        label=boxes[b, :n, 4].numpy().astype(np.int64)))
    return out


def _run_train(monkeypatch, model, data, tmp_path, lr, eager=False):
    """train() with the reference keywords for one step; returns the trainer's per-image losses,
    targets, head outputs and the sample order the loop drew."""
    from cvlite import train_fcos as tf_mod
    rec = {}
    base = tf_mod.FCOSTrainer

    class Spy(base):
        def __init__(self, *a, **k):
            if eager:
                k["use_graph"] = False
            super().__init__(*a, **k)

        def step(self):
            out = super().step()
            rec["losses"] = out.detach().clone()
            rec["targets"] = self.targets.detach().clone()
            rec["outputs"] = tuple(t.detach().clone() for t in self.outputs)
            return out
    monkeypatch.setattr(tf_mod, "FCOSTrainer", Spy)
    np.random.seed(SEED)
    idx = np.random.choice(len(data), size=B, replace=False)          # the loop's own draw
    np.random.seed(SEED)
    losses = []
    tf_mod.train(data, losses, model, B, tf_mod.SGD(learning_rate=lr, momentum=0.9), "", None, 0, 1,
                 init_lr=lr, min_lr=1e-5, decay_step=1000, decay_rate=0.99, display_step=1, step_save=1,
                 step_cool=1000, weight_decay=0.0, gradient_clip=1.0,
                 save_loss_file=str(tmp_path / "train_losses.csv"))
    torch.cuda.synchronize()
    assert len(losses) == 1 and losses[0][0] == 1 and np.isfinite(losses[0][1])
    return rec, idx


def _check_targets(rec, data, idx):
    tg = rec["targets"].cpu().numpy()
    for k, i in enumerate(idx):
        outs, _ = fcos_ref.format_data(_gt(data, i), np.array([S, S], np.float32), C, img_pad=(S, S))
        np.testing.assert_array_equal(tg[k], fcos_ref.pack_targets(outs))
    return torch.from_numpy(tg)


def _flat_rel(a, b, keys):
    n = d = 0.0
    for k in keys:
        n += float((a[k].double() - b[k].double()).norm() ** 2)
        d += float(b[k].double().norm() ** 2)
    return math.sqrt(n / max(d, 1e-300))


def _gt(data, i):
    s = data[i]
    return np.concatenate([s["bbox"], s["label"].astype(np.float32)[:, None]], 1)


def test_configs0_train_loop_fp32_parity(monkeypatch, tmp_path):
    from cvlite import fcos
    monkeypatch.setenv("CVL_PRECISION", "fp32")
    lr = 5e-4
    model = fcos.build_model(C)
    net = model.net
    assert net.store.act == torch.float32
    for k in net.store.offsets:                      # damped residual branches (module docstring)
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(0.25)
    p0 = net.store.state_dict()
    names = list(p0)
    data = _samples()
    rec, idx = _run_train(monkeypatch, model, data, tmp_path, lr)
    tg = _check_targets(rec, data, idx)
    x = torch.from_numpy(np.stack([data[i]["image"] for i in idx]))
    P64 = {k: v.clone().double() for k, v in p0.items()}
    M64 = {k: torch.zeros_like(v) for k, v in P64.items()}
    P32 = {k: v.clone() for k, v in p0.items()}
    M32 = {k: torch.zeros_like(v) for k, v in p0.items()}
    l64 = []
    norm64 = model_ref.train_step_reference(P64, M64, x.double(), tg.double(), C, lr, dtype=torch.float64,
                                            losses_out=l64)
    l64 = torch.stack(l64)
    model_ref.train_step_reference(P32, M32, x, tg, C, lr)
    st = net.store
    mom = {k: st.mom[st.offsets[k][0]:st.offsets[k][0] + st.offsets[k][1]].view(st.offsets[k][2]).cpu()
           for k in names}
    par = {k: st.p(k).detach().cpu() for k in names}
    e_mom, e_mom32 = _flat_rel(mom, M64, names), _flat_rel(M32, M64, names)
    e_par = _flat_rel(par, P64, names)
    got = rec["losses"].cpu().double()
    e_loss = float(((got - l64).abs() / l64.abs().clamp(min=1e-12)).max())
    print("configs[0] fp32: grad norm %.6e; momentum rel-L2 gpu-vs-fp64 %.2e (cpu fp32 %.2e); params %.2e; "
          "losses max rel %.2e" % (norm64, e_mom, e_mom32, e_par, e_loss))
    assert e_loss <= LOSS_RTOL_F32
    assert e_mom <= max(MOM_RTOL, NOISE_X * e_mom32)
    assert e_par <= 1e-4
    assert not any(torch.equal(par[k], p0[k]) for k in names if k.endswith("kernel:0") and "cls_layer_1" in k)


def test_configs0_train_loop_bf16_launch_parity(monkeypatch, tmp_path):
    from launch_parity import LaunchParity
    from cvlite import fcos
    monkeypatch.delenv("CVL_PRECISION", raising=False)
    lr = 5e-4
    model = fcos.build_model(C)
    net = model.net
    assert net.store.act == torch.bfloat16
    w0 = net.store.flat.clone()
    data = _samples()
    with LaunchParity(imgs=None) as lp:
        rec, idx = _run_train(monkeypatch, model, data, tmp_path, lr, eager=True)
    bad = lp.failures()
    print("configs[0] bf16 launch parity: %d checks, %d failures" % (len(lp.records), len(bad)))
    assert not bad, "\n".join(r.line() for r in bad[:40])
    assert not lp.unchecked_calls(), lp.unchecked_calls()
    assert len(lp.records) > 500
    _check_targets(rec, data, idx)
    tg = rec["targets"].cpu().numpy()
    reg, cls = (t.cpu().float().numpy() for t in rec["outputs"])
    got = rec["losses"].cpu().double().numpy()
    for k in range(B):
        pred = np.concatenate([reg[k, :, :5], cls[k, :, :C]], 1)
        preds, o = [], 0
        for s in (64, 32, 16, 8, 4):
            preds.append(pred[o:o + s * s].reshape(1, s, s, 5 + C))
            o += s * s
        outs, _ = fcos_ref.format_data(_gt(data, idx[k]), np.array([S, S], np.float32), C, img_pad=(S, S))
        ref = np.array(fcos_ref.model_loss(outs, preds), np.float64)
        np.testing.assert_allclose(got[k], ref, rtol=2e-5, atol=1e-4)
    assert torch.isfinite(net.store.flat).all() and float((net.store.flat - w0).abs().max()) > 0
