"""Time the FPN P7 conv's weight gradient (3x3 s2 256->256, 8x8 -> 4x4, relu on load; the generic
conv_wgrad_kernel) alone, graph-replayed, under settings: c7_probe.py "" "CVL_WG_BR128=1" ...
Variants of the launch itself: relu_in off, and the same shapes at stride 1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from cvlite import ops_nn as nn, _lib  # noqa: E402
from p_probe import timed  # noqa: E402


def main():
    L = _lib.load()
    B = 16
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn((B, 8, 8, 256), generator=g).to(torch.bfloat16).cuda()
    dy = torch.randn((B, 4, 4, 256), generator=g).to(torch.bfloat16).cuda()
    wf = torch.zeros((256, 9 * 256), dtype=torch.bfloat16, device="cuda")
    dw = torch.zeros((3, 3, 256, 256), dtype=torch.float32, device="cuda")
    x1 = torch.randn((B, 4, 4, 256), generator=g).to(torch.bfloat16).cuda()
    for stt in sys.argv[1:] or [""]:
        kv = [t.split("=", 1) for t in stt.split()]
        for k, v in kv:
            os.environ[k] = v
        res = []
        for name, st, relu, src, Hs in (("s2 relu", 2, True, x, 8), ("s2", 2, False, x, 8), ("s1 4x4", 1, False, x1, 4)):
            d = nn.make_desc(nn.FWD, B, 256, 3, 3, st, 0 if st == 2 else 1, 0 if st == 2 else 1, 256, 256, 256,
                             [nn.seg(4, 4, Hs, Hs, wf, None)], relu_in=relu)
            us = timed(lambda: nn.conv_wgrad(d, src, dy, dw))
            kn = L.cvl_conv_kernel_name(L.cvl_conv_igemm_last_kernel()).decode().split(" ")[0]
            res.append("%s %.1f us (%s)" % (name, us, kn))
        for k, _ in kv:
            del os.environ[k]
        print("%-24s %s" % (stt or "default", "  |  ".join(res)), flush=True)


if __name__ == "__main__":
    main()
