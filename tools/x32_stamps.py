"""Per-workgroup timeline of the tower conv (X32, CVL_X_ABLATE 256|8|extra: stamps in dst, no epilogue)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    B, H, W = 16, 512, 512
    shapes, off, P = net.layout(B, H, W)
    g = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn((2 * B * P, 256), generator=g) * 0.5).to(torch.bfloat16).cuda()
    d = net.cls_tower[1].fwd_desc(B, net._pair_segs(1, B, shapes, off, P, fwd=True), ld_dst=256)
    for extra in [int(x) for x in sys.argv[1:]] or [0]:
        dst = torch.zeros_like(src)
        os.environ["CVL_X_ABLATE"] = str(256 | 8 | extra)
        # >= 2 s of back-to-back launches first: the clock the chip holds under this load (DVFS)
        t_end = time.time() + 2.0
        while time.time() < t_end:
            for _ in range(50):
                nn.conv_igemm(d, src, dst)
            torch.cuda.synchronize()
        s = dst.view(torch.int64).view(-1, 4)[:682].cpu().double()
        t0 = s[:, 0].min()
        pro = (s[:, 1] - s[:, 0]) / 100.0
        loop = (s[:, 2] - s[:, 1]) / 100.0
        ent = ((s[:, 0] - t0) / 100.0).sort().values
        end = ((s[:, 2] - t0) / 100.0).max()
        nk = d.Cin * d.KH * d.KW // 32
        ghz = (s[:, 3] / (s[:, 2] - s[:, 1]) * 0.1).median()     # shader ticks / 100 MHz wall ticks
        print("ablate %d: span %.1f us | prologue median %.2f loop median %.1f us (%.3f us per K-tile, nk %d) | "
              "in-kernel clock %.3f GHz | entry at ranks 0/255/256/511/512/681: %s"
              % (extra, end, pro.median(), loop.median(), loop.median() / nk, nk, ghz,
                 [round(float(ent[i]), 1) for i in (0, 255, 256, 511, 512, 681)]))
    os.environ.pop("CVL_X_ABLATE", None)


if __name__ == "__main__":
    main()
