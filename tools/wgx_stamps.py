"""Per-workgroup timeline of the 2-D weight-gradient kernel (conv_wgrad_x) on every launch it takes
in one FCOS training step (configs[1], 512x512 bs 16): entry spread, prologue (first DMA steps
landed), main loop, epilogue (slab / dW stores), and the kernel span, from in-kernel wall-clock
stamps (CVL_WGX_STAMPS=1, cvl_debug_wgx_stamps).  usage: wgx_stamps.py [--bs 16]"""
import argparse
import collections
import ctypes
import os
import sys

os.environ["CVL_WGX_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from conv_table import desc_key, describe  # noqa: E402
from cvlite import _lib, ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402
from cvlite.train_fcos import FCOSTrainer, synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=16)
    args = ap.parse_args()
    B, H = args.bs, 512
    net = FCOSNet(20, device=torch.device("cuda"), seed=0)
    tr = FCOSTrainer(net, B, (H, H), use_graph=False)
    tr.load_batch(*synthetic_batch(B, H, H, 20, seed=1234, device="cuda"))
    tr.step()
    torch.cuda.synchronize()
    calls = collections.OrderedDict()
    counts = collections.Counter()
    orig = (nn.conv_wgrad, nn.conv_wgrad_grouped)

    def wgrad(desc, x, dy, dw, beta=0.0):
        k = desc_key("wgrad", desc)
        counts[k] += 1
        calls.setdefault(k, (lambda: orig[0](desc, x, dy, dw, beta), desc, 1))
        return orig[0](desc, x, dy, dw, beta)

    def wgrad_g(desc, x, dy, dws, beta=0.0):
        k = desc_key("wgrad_g", desc)
        counts[k] += 1
        calls.setdefault(k, (lambda: orig[1](desc, x, dy, dws, beta), desc, len(dws)))
        return orig[1](desc, x, dy, dws, beta)

    nn.conv_wgrad, nn.conv_wgrad_grouped = wgrad, wgrad_g
    tr.step()
    torch.cuda.synchronize()
    nn.conv_wgrad, nn.conv_wgrad_grouped = orig
    lib = _lib.load()
    buf = (ctypes.c_uint64 * (16384 * 4))()
    phases = []
    print("| launch | per step | WGs | entry spread us | prologue us | loop us | epilogue us | WG total us | span us |")
    print("|---|---|---|---|---|---|---|---|---|")
    for key, (replay, d, ng) in calls.items():
        replay()
        if lib.cvl_conv_igemm_last_kernel() != 11:          # CVL_CK_WG_X
            continue
        for _ in range(3):
            replay()
        torch.cuda.synchronize()
        n = lib.cvl_debug_wgx_stamps(buf, 16384)
        if n <= 0:
            continue
        s = torch.tensor(list(buf[:n * 4]), dtype=torch.float64).view(n, 4)
        t0 = s[:, 0].min()
        us = lambda v: float(v) / 100.0                      # 100 MHz wall clock
        row = (describe("wgrad", d, ng), counts[key], n, us((s[:, 0] - t0).max()),
               us((s[:, 1] - s[:, 0]).median()), us((s[:, 2] - s[:, 1]).median()), us((s[:, 3] - s[:, 2]).median()),
               us((s[:, 3] - s[:, 0]).median()), us(s[:, 3].max() - t0))
        print("| %s | %d | %d | %.1f | %.2f | %.1f | %.2f | %.1f | %.1f |" % row)
        if hasattr(lib, "cvl_debug_wgx_phase"):
            pb = (ctypes.c_uint64 * (n * 64))()
            if lib.cvl_debug_wgx_phase(pb, n) > 0:
                ph = torch.tensor(list(pb[:n * 64]), dtype=torch.float64).view(n, 8, 8)
                steps = ph[:, :, 5].clamp(min=1)
                per = ph[:, :, :5] / steps[..., None]               # cycles per step, per wave
                for grp in (0, 1):
                    m = per[ph[:, :, 7] == grp].median(0).values
                    phases.append("| %s | g%d | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f |" % (
                        describe("wgrad", d, ng), grp, m[0], m[1], m[2], m[3], m[4], float(m.sum())))
    if phases:
        print()
        print("Per-step loop phases (shader cycles, median wave of each group): data wait | LDS segment "
              "(ring writes, loads, fragment reads landed) | barrier 1 | MFMA issue | barrier 2 | sum")
        print()
        print("| launch | group | wait | LDS | bar1 | MFMA | bar2 | sum |")
        print("|---|---|---|---|---|---|---|---|")
        for r in phases:
            print(r)


if __name__ == "__main__":
    main()
