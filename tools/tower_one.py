"""Runs ONE conv kernel variant on the paired FCOS tower layer (bs 16, 512x512) N times, for
rocprofv3 --pmc passes.  usage: [env knobs] python tools/tower_one.py [iters] [fwd|dgrad]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    mode = sys.argv[2] if len(sys.argv) > 2 else "fwd"
    B, H, W = 16, 512, 512
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    shapes, off, P = net.layout(B, H, W)
    g = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn((2 * B * P, 256), generator=g) * 0.5).to(torch.bfloat16).cuda()
    d = net.cls_tower[1].fwd_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=True), ld_dst=256) if mode == "fwd" \
        else net.cls_tower[1].dgrad_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=False), ld_dst=256)
    dst = torch.empty_like(src)
    nn.conv_igemm(d, src, dst)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        nn.conv_igemm(d, src, dst)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    from cvlite import _lib
    L = _lib.load()
    M = 2 * B * P
    print("done", iters, mode, L.cvl_conv_kernel_name(L.cvl_conv_igemm_last_kernel()).decode(),
          "%.1f us  %.0f TFLOP/s" % (us, 2.0 * M * 256 * 2304 / us / 1e6))


if __name__ == "__main__":
    main()
