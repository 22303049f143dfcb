"""Teacher-forced per-launch parity of ONE real production training step at the BASELINE.json
geometries: configs[1] FCOS R50-FPN 512x512, configs[3] CenterNet hourglass
512x512 (sub-batch 2), configs[4] RetinaNet R50-FPN 640x640 C = 80.

The trainer runs eagerly (use_graph=False: the same Python calls the production HIP graphs
capture -> the same kernels, planner choices, split-K / deferred-reduction paths and fused
epilogues).  tests/launch_parity.py wraps every device op: for each launch it snapshots the GPU's
own inputs, lets the kernel run, and compares the result with float64 torch on those inputs --
forward, data gradient and weight gradient of every conv (incl. the fused BN-statistics,
BN-backward-first-pass and residual epilogues), every BN / pool / up-sample / bias / optimizer /
re-pack launch.  bf16 outputs rel-L2 <= 1e-2, fp32 <= 1e-4 (cancelling reductions normalised by
their |terms|), pool values / argmax / im2col / packs bit-exact.  It also asserts that every C
entry point the step launched went through a checked wrapper.

Batch: the configs' own (FCOS 16, CenterNet 8, RetinaNet 8; CVL_TF_BS overrides) -- the tile
planner picks kernels by problem size, so only the full batch exercises the shipped dispatch (X32
towers, split-K choices).  Every image of every launch is compared (CVL_TF_IMGS=<n> restricts the
forward / data-gradient references to n images); the float64 references run on the GPU, a few
seconds per step."""
import os

import pytest
import torch

from launch_parity import LaunchParity

pytestmark = pytest.mark.gpu


def _imgs():
    v = os.environ.get("CVL_TF_IMGS", "all")
    return None if v == "all" else int(v)


def _report(lp, tag):
    txt = lp.table()
    kinds = sorted({r.kernel for r in lp.records if r.kernel})
    head = "%s: %d checks, %d failures; conv kernels seen: %s\n" % (tag, len(lp.records), len(lp.failures()),
                                                                   ", ".join(kinds))
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "launch_parity_%s.txt" % tag), "w") as f:
            f.write(head + txt + "\n")
    print(head)
    bad = lp.failures()
    assert not bad, "teacher-forced launch parity failures:\n" + "\n".join(r.line() for r in bad[:60])
    unchecked = lp.unchecked_calls()
    assert not unchecked, "launches outside the checked wrappers: %r" % unchecked
    return kinds


def test_fcos_step_launch_parity_configs1():
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    C, S = 20, 512
    B = int(os.environ.get("CVL_TF_BS", 16))
    net = FCOSNet(C, seed=0)
    tr = FCOSTrainer(net, B, (S, S), use_graph=False)
    tr.load_batch(*synthetic_batch(B, S, S, C, seed=2024))
    with LaunchParity(imgs=_imgs()) as lp:
        tr.step()
    kinds = _report(lp, "fcos_512_bs%d" % B)
    # the shipped kernels of configs[1] took part (the dispatch is the production one)
    for k in ("X32", "P", "H64", "WG_X"):
        assert any(k == x or x.startswith(k) for x in kinds), (k, kinds)


def test_centernet_step_launch_parity_configs3():
    from cvlite.hourglass_net import HourglassNet
    from cvlite.train_centernet import CenterNetTrainer, synthetic_batch
    C, S = 20, 512
    B = int(os.environ.get("CVL_TF_BS", 8))
    net = HourglassNet(C, seed=0)
    tr = CenterNetTrainer(net, B, (S, S), sub_batch_sz=2, n_max=16, use_graph=False)
    tr.load_batch(*synthetic_batch(B, S, S, C, n_max=16, seed=77))
    with LaunchParity(imgs=_imgs()) as lp:
        tr.step()
    _report(lp, "centernet_512_bs%d" % B)


def test_retinanet_step_launch_parity_configs4():
    from cvlite.retinanet import RetinaNet
    from cvlite.train_retinanet import RetinaTrainer, synthetic_coco_batch
    C, S = 80, 640
    B = int(os.environ.get("CVL_TF_BS", 8))
    rn = RetinaNet(C, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
    tr = RetinaTrainer(rn.model, rn, B, S, n_max=50, use_graph=False)
    tr.load_candidates(*synthetic_coco_batch(3 * B, S, C, n_max=50, seed=4321))
    with LaunchParity(imgs=_imgs()) as lp:
        tr.step()
    _report(lp, "retinanet_640_bs%d" % B)


def test_launch_parity_catches_a_wrong_kernel(monkeypatch):
    """The harness is not vacuous: a perturbed conv output is flagged."""
    from cvlite import ops_nn as nn
    from cvlite.layers import Conv, ParamStore
    st = ParamStore()
    conv = Conv(st, "c", 3, 64, 64)
    st.finalize(torch.device("cuda", 0), seed=1)
    conv.pack()
    x = torch.randn((2, 32, 32, 64), device="cuda").to(torch.bfloat16)
    orig = nn.conv_igemm

    def broken(desc, src, dst, stats=None):
        orig(desc, src, dst, stats)
        dst.view(-1)[::97] += 0.5
    monkeypatch.setattr(nn, "conv_igemm", broken)
    with LaunchParity() as lp:
        conv.fwd(x, 2, 32, 32)
    torch.cuda.synchronize()
    assert lp.failures() and lp.records[0].op == "conv_igemm"


@pytest.mark.parametrize("opts", [dict(n_stacks=2), dict(seperable=False, norm_order="norm_last"),
                                  dict(batch_norm=False)], ids=["stacks2", "dense-normlast", "nobn"])
def test_centernet_build_options_launch_parity(opts):
    """The non-default tf_centernet_hourglass.build_model options, every launch of one training step
    (256x256, bs 4, sub-batch 2) teacher-forced against float64."""
    from cvlite.hourglass_net import HourglassNet
    from cvlite.train_centernet import CenterNetTrainer, synthetic_batch
    C, S, B = 20, 256, 4
    net = HourglassNet(C, seed=0, n_filters=64, **opts)
    tr = CenterNetTrainer(net, B, (S, S), sub_batch_sz=2, n_max=16, use_graph=False)
    tr.load_batch(*synthetic_batch(B, S, S, C, n_max=16, seed=78))
    with LaunchParity(imgs=_imgs()) as lp:
        tr.step()
    _report(lp, "centernet_opts_%s" % "_".join("%s%s" % kv for kv in sorted(opts.items())))
