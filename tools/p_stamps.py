"""Per-workgroup wall time of the persistent 1x1 kernel (CVL_P_ABLATE=10 + extra bits: stamps in dst,
no stores) vs the launch time: is the time inside the workgroups or in their start-up / tail?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn  # noqa: E402
from p_probe import CASES, timed  # noqa: E402


def main():
    extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    gen = torch.Generator(device="cpu").manual_seed(0)
    for (B, H, Cin, Cout, st, stats) in CASES:
        x = torch.randn((B, H, H, Cin), generator=gen).to(torch.bfloat16).cuda()
        w = (torch.randn((Cout, Cin), generator=gen) * Cin ** -0.5).to(torch.bfloat16).cuda()
        y = torch.zeros((B, H, H, Cout), dtype=torch.bfloat16, device="cuda")
        sts = nn.bn_acc(B, Cout, "cuda")
        d = nn.make_desc(nn.FWD, B, Cin, 1, 1, 1, 0, 0, Cout, Cout, Cout, [nn.seg(H, H, H, H, w, None)])
        os.environ["CVL_P_ABLATE"] = str(10 | extra)
        us = timed(lambda: nn.conv_igemm(d, x, y, sts))
        s = y.view(torch.int64).view(-1, 4)[:256].cpu().double()
        n = int((s[:, 0] > 0).sum())
        s = s[:n]
        t0 = s[:, 0].min()
        dur = (s[:, 1] - s[:, 0]) / 100.0
        start = (s[:, 0] - t0) / 100.0
        print("fwd 1x1 %d->%d @ %d: launch %.1f us | %d WGs, K-tiles/WG %d, WG time median %.1f max %.1f, "
              "start spread %.1f us -> %.2f us per K-tile" % (Cin, Cout, H, us, n, int(s[0, 2]), dur.median(), dur.max(),
                                                           start.max(), dur.median() / max(1, int(s[0, 2]))))
    os.environ.pop("CVL_P_ABLATE", None)


if __name__ == "__main__":
    main()
