"""Per-workgroup timeline of the stem forward kernel (cvl_stem_conv7x7s2) at the FCOS geometry
(bs 16, 512x512) from in-kernel stamps (CVL_STEM_STAMPS=1, cvl_debug_stem_stamps): entry spread,
prologue (ring zeroed + first 7 image rows), the 8 output rows, the statistics flush, and the
shader-clock split of the rows into MFMA phase / epilogue (bias, bf16, stats, stores) / ring
refill (the wait for the next rows' loads + LDS stores + barriers).  usage: stem_stamps.py"""
import ctypes
import os
import sys

os.environ["CVL_STEM_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cvlite import _lib, ops_nn as nn  # noqa: E402


def main():
    B, H = 16, 512
    img = torch.rand((B, H, H, 3), device="cuda") * 2 - 1
    wf = (torch.randn((64, 168), device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.zeros(64, device="cuda")
    z = torch.empty((B, 256, 256, 64), dtype=torch.bfloat16, device="cuda")
    for _ in range(3):
        st = nn.bn_acc(B, 64, "cuda")
        nn.stem_conv7x7s2(img, wf, bias, z, st)
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    n = _lib.load().cvl_debug_stem_stamps(buf.ctypes.data_as(ctypes.c_void_p), 4096)
    s = buf[:n].astype(np.float64)
    wall = 100.0                                              # wall clock ticks per us (100 MHz)
    t0 = s[:, 0].min()
    span = (s[:, 3].max() - t0) / wall
    pro = ((s[:, 1] - s[:, 0]) / wall).mean()
    rows = ((s[:, 2] - s[:, 1]) / wall).mean()
    fin = ((s[:, 3] - s[:, 2]) / wall).mean()
    cyc = s[:, 4] + s[:, 5] + s[:, 6]
    clk = (cyc / ((s[:, 2] - s[:, 1]) / wall)).mean()        # shader ticks per us over the rows
    print("stem fwd: %d WGs, span %.1f us, entry spread %.1f us; per WG: prologue %.1f, rows %.1f, "
          "stats+exit %.1f us; rows split (shader clock %.0f MHz): MFMA phase %.1f, epilogue %.1f, refill %.1f us"
          % (n, span, (s[:, 0].max() - t0) / wall, pro, rows, fin, clk,
             (s[:, 4] / clk).mean(), (s[:, 5] / clk).mean(), (s[:, 6] / clk).mean()))


if __name__ == "__main__":
    main()
