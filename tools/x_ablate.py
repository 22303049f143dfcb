"""Ablation timings of the X conv kernel on the paired FCOS tower layer (forward): CVL_X_ABLATE
bits 1 = no A traffic, 2 = no B traffic, 4 = no MFMA, 8 = no barriers, 16 = no vmcnt waits,
32 = no LDS-DMA instructions, 64 = no LDS fragment reads
(results are wrong for every non-zero setting: timing insight only).  Interleaved rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402
from tower_ab import run  # noqa: E402

SETTINGS = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "0,1,2,3,4,7,8,16,24".split(","))]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B, H, W = 16, 512, 512
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    shapes, off, P = net.layout(B, H, W)
    g = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn((2 * B * P, 256), generator=g) * 0.5).to(torch.bfloat16).cuda()
    fd = net.cls_tower[1].fwd_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=True), ld_dst=256)
    flops = 2.0 * 2 * B * P * 256 * 9 * 256
    dst = torch.empty_like(src)
    res = {k: [] for k in SETTINGS}
    for r in range(rounds):
        for k in SETTINGS:
            os.environ["CVL_X_ABLATE"] = str(k)
            res[k].append(run(lambda: nn.conv_igemm(fd, src, dst), 10))
    os.environ.pop("CVL_X_ABLATE")
    for k in SETTINGS:
        t = sorted(res[k])[len(res[k]) // 2]
        print("ablate %2d: %.4f ms  (%.0f TFLOP/s equiv)" % (k, t, flops / t / 1e9), flush=True)


if __name__ == "__main__":
    main()
