"""A/B of the 256x256 conv kernels on the paired FCOS tower layer (both towers, 5 levels, bs 16,
512x512: M = 174,592, N = 256, K = 2,304), forward and data gradient, in ONE process with
interleaved rounds (HIP events): the 8-phase X kernel vs the L kernel (CVL_CONV_NO_X=1); also
prints the max |X - L| of the outputs.  usage: python tools/tower_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import _lib, ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402

VARIANTS = {"L256": {"CVL_CONV_NO_X": "1"}, "X": {"CVL_CONV_NO_X32": "1"}, "X32": {}}
KEYS = ("CVL_CONV_NO_X", "CVL_CONV_NO_X32")


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
    g = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn((2 * B * P, 256), generator=g) * 0.5).to(torch.bfloat16).cuda()
    fd = net.cls_tower[1].fwd_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=True), ld_dst=256)
    dd = net.cls_tower[1].dgrad_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=False), ld_dst=256)
    flops = 2.0 * 2 * B * P * 256 * 9 * 256
    outs = {}
    lib = _lib.load()
    for name, env in VARIANTS.items():
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        for m, d in (("fwd", fd), ("dgrad", dd)):
            dst = torch.empty_like(src)
            nn.conv_igemm(d, src, dst)
            torch.cuda.synchronize()
            outs[(name, m)] = dst
            print(name, m, "->", lib.cvl_conv_kernel_name(lib.cvl_conv_igemm_last_kernel()).decode(), flush=True)
    for m in ("fwd", "dgrad"):
        for v in VARIANTS:
            a, b = outs[("L256", m)].float(), outs[(v, m)].float()
            print("%s max|%s-L256| %.4g (max|L| %.3g)" % (m, v, float((a - b).abs().max()), float(a.abs().max())),
                  flush=True)
    res = {k: {"fwd": [], "dgrad": []} for k in VARIANTS}
    dst = torch.empty_like(src)
    for r in range(rounds):
        for name, env in VARIANTS.items():
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            res[name]["fwd"].append(run(lambda: nn.conv_igemm(fd, src, dst), 10))
            res[name]["dgrad"].append(run(lambda: nn.conv_igemm(dd, src, dst), 10))
    for name in VARIANTS:
        for m in ("fwd", "dgrad"):
            v = sorted(res[name][m])
            t = v[len(v) // 2]
            print("%-6s %-5s median %.4f ms (min %.4f)  %.0f TFLOP/s  frac %.3f" % (
                name, m, t, v[0], flops / t / 1e9, flops / t / 1e9 / 2500.0), flush=True)


if __name__ == "__main__":
    main()
