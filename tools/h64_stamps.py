"""Per-workgroup timeline of the H64 kernel (conv_igemm_h.hip) on the backbone 3x3 forward launches
at the FCOS geometry (bs 16, 512x512: conv2_x..conv5_x 3x3 units) from in-kernel stamps
(CVL_H_STAMPS=1, cvl_debug_h_stamps): entry spread, prologue, the tile loop, and the shader-clock
split of a workgroup's time into tap loops (LDS fragment reads + MFMA + DMA issue), the per-block
wait + barrier (DMA latency not hidden by the taps), and the epilogues.  usage: h64_stamps.py"""
import ctypes
import os
import sys

os.environ["CVL_H_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import _lib, ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    lib = _lib.load()
    net = FCOSNet(bench.NUM_CLASSES, device=torch.device("cuda", 0), seed=0)
    B, h, w = 16, 128, 128
    g = torch.Generator(device="cpu").manual_seed(3)
    for si, stage in enumerate(net.backbone.stages):
        if si > 0:
            h, w = h // 2, w // 2
        conv = stage[-1].c2.conv
        C = conv.cin
        x = torch.randn((B, h, w, C), generator=g).to(torch.bfloat16).cuda()
        y = torch.zeros((B, h, w, conv.cout), dtype=torch.bfloat16, device="cuda")
        fd = conv.fwd_desc(B, [nn.seg(h, w, h, w, conv.wf, conv.bias_arg())], ld_dst=conv.cout)
        st = nn.bn_acc(B, conv.cout, "cuda")
        report(lib, "stage %d fwd 3x3 %d->%d @ %dx%d" % (si, C, conv.cout, h, w), lambda: nn.conv_igemm(fd, x, y, st))
        # the fused data gradient + next BN's backward first pass (conv.dgrad with bn_next)
        z = torch.randn((B, h, w, C), generator=g).to(torch.bfloat16).cuda()
        mr = torch.stack([torch.zeros(B, C), torch.ones(B, C)], -1).cuda()
        ga, be = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        dx = torch.empty((B, h, w, C), dtype=torch.bfloat16, device="cuda")
        sums = nn.bn_acc(B, C, "cuda")
        dd = conv.dgrad_desc(B, [nn.seg(h, w, h, w, conv.wd)], ld_dst=C)
        report(lib, "stage %d dgrad+bnsum 3x3 %d->%d @ %dx%d" % (si, conv.cout, C, h, w),
               lambda: nn.conv_igemm_dgrad_bnsum(dd, y, dx, z, mr, ga, be, sums))


def report(lib, name, launch):
    wall = 100.0                                              # wall clock ticks per us (100 MHz)
    lib.cvl_debug_h_stamps(None, -1)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / 20
    if True:
        buf = np.zeros((4096, 8), dtype=np.uint64)
        n = lib.cvl_debug_h_stamps(buf.ctypes.data_as(ctypes.c_void_p), 4096)
        if n <= 0:
            print("%s: not an unsplit H64 launch (%.1f us)" % (name, us))
            return
        ph = np.stack([(buf[:n, 2] >> np.uint64(16 * k)) & np.uint64(0xffff) for k in range(4)], 1).astype(np.float64)
        s = buf[:n].astype(np.float64)
        t0 = s[:, 0].min()
        span = (s[:, 3].max() - t0) / wall
        pro = ((s[:, 1] - s[:, 0]) / wall).mean()
        loop = ((s[:, 3] - s[:, 1]) / wall).mean()
        cyc = s[:, 4] + s[:, 5] + s[:, 6]
        clk = (cyc / np.maximum((s[:, 3] - s[:, 1]) / wall, 1e-3)).mean()   # shader ticks per us
        print("%s: %.1f us/launch (events), %d WGs x %.1f tiles, span %.1f us, entry "
              "spread %.1f us; per WG: prologue %.1f, tiles %.1f us; split (shader clock %.0f MHz): taps %.1f, "
              "block wait+barrier %.1f, epilogue %.1f us"
              % (name, us, n, s[:, 7].mean(), span, (s[:, 0].max() - t0) / wall, pro, loop, clk,
                 (s[:, 4] / clk).mean(), (s[:, 5] / clk).mean(), (s[:, 6] / clk).mean()))
        tiles = np.maximum(s[:, 7], 1)[:, None]
        print("   epilogue per tile (us): rounding+stats+barrier %.2f, C image+combine %.2f, stores(+sums) %.2f, "
              "sums reduction %.2f" % tuple((ph / tiles / clk).mean(0)))


if __name__ == "__main__":
    main()
