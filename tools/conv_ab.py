"""A/B of the large-tile conv variants on the FCOS tower shape (fwd + dgrad, all 5 levels, bs=16,
512x512) in ONE process, interleaved rounds (HIP events): 128-wide tile vs 256-wide tile, MFMA
priority on/off.  usage: python tools/conv_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402

VARIANTS = {"bn128": {"CVL_CONV_NO_256": "1"}, "bn128_noprio": {"CVL_CONV_NO_256": "1", "CVL_CONV_NO_PRIO": "1"},
            "bn256": {"CVL_CONV_L256_MIN_TILES": "1"}, "bn256_noprio": {"CVL_CONV_L256_MIN_TILES": "1", "CVL_CONV_NO_PRIO": "1"}}
KEYS = ("CVL_CONV_NO_256", "CVL_CONV_NO_PRIO", "CVL_CONV_L256_MIN_TILES")


def run(fn, iters):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    B, H, W = 16, 512, 512
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    shapes, off, P = net.layout(B, H, W)
    conv = net.cls_tower[1]
    g = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn((B * P, 256), generator=g) * 0.5).to(torch.bfloat16).cuda()
    dst = torch.empty_like(src)
    fd = conv.fwd_desc(B, net._tower_segs(conv, B, shapes, off), ld_dst=256)
    dd = conv.dgrad_desc(B, net._tower_segs(conv, B, shapes, off, wf=False), ld_dst=256)
    flops = 2.0 * B * P * 256 * 9 * 256
    res = {k: {"fwd": [], "dgrad": []} for k in VARIANTS}
    for r in range(rounds):
        for name, env in VARIANTS.items():
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            res[name]["fwd"].append(run(lambda: nn.conv_igemm(fd, src, dst), 10))
            res[name]["dgrad"].append(run(lambda: nn.conv_igemm(dd, src, dst), 10))
    for name in VARIANTS:
        for m in ("fwd", "dgrad"):
            t = sorted(res[name][m])[len(res[name][m]) // 2]
            print("%-14s %-5s median %.4f ms  %.0f TFLOP/s" % (name, m, t, flops / t / 1e9), flush=True)


if __name__ == "__main__":
    main()
