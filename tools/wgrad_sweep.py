"""Weight-gradient kernel / split sweep on the FCOS step's backbone wgrad shapes (bs 16, 512x512):
for each shape, the default dispatch, the L / 128-tile kernels (CVL_WGRAD_NO_X), the 128-tile
kernel alone (+ CVL_WGRAD_NO_L), and the X kernel at forced split counts (CVL_WGX_SPLITS).  Times
are HIP-event medians of 3 rounds x 10 launches, one process (knobs are read per launch).
usage: wgrad_sweep.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import _lib  # noqa: E402
from cvlite.layers import Conv, ParamStore  # noqa: E402

BF = torch.bfloat16
# (B, H, W, cin, cout, k, stride) of the backbone wgrad launches (r02i conv table), forward geometry
SHAPES = [(16, 32, 32, 256, 256, 3, 1), (16, 32, 32, 1024, 256, 1, 1), (16, 32, 32, 256, 1024, 1, 1),
          (16, 64, 64, 128, 512, 1, 1), (16, 64, 64, 128, 128, 3, 1), (16, 128, 128, 64, 64, 3, 1),
          (16, 128, 128, 64, 256, 1, 1), (16, 64, 64, 512, 128, 1, 1), (16, 16, 16, 512, 512, 3, 1),
          (16, 16, 16, 512, 2048, 1, 1), (16, 16, 16, 2048, 512, 1, 1), (16, 128, 128, 256, 64, 1, 1)]
VARIANTS = [("default", {}), ("noX", {"CVL_WGRAD_NO_X": "1"}), ("old", {"CVL_WGRAD_NO_X": "1", "CVL_WGRAD_NO_L": "1"})]
VARIANTS += [("X s%d" % s, {"CVL_WGX_SPLITS": str(s)}) for s in (4, 8, 16, 32, 64)]
KEYS = ("CVL_WGRAD_NO_X", "CVL_WGRAD_NO_L", "CVL_WGX_SPLITS")


def timed(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    lib = _lib.load()
    for (B, H, W, cin, cout, k, s) in SHAPES:
        st = ParamStore()
        c = Conv(st, "c", k, cin, cout, stride=s)
        st.finalize("cuda", 0)
        c.pack()
        Ho, Wo, _, _ = c.out_hw(H, W)
        x = torch.randn((B, H, W, cin), device="cuda").to(BF)
        dy = torch.randn((B, Ho, Wo, cout), device="cuda").to(BF)
        fl = 2.0 * B * Ho * Wo * cout * k * k * cin
        res = {name: [] for name, _ in VARIANTS}
        kern = {}
        for _ in range(rounds):
            for name, env in VARIANTS:
                for key in KEYS:
                    os.environ.pop(key, None)
                os.environ.update(env)
                res[name].append(timed(lambda: c.wgrad(x, dy, B, H, W, bias=False)))
                kern[name] = lib.cvl_conv_kernel_name(lib.cvl_conv_igemm_last_kernel()).decode().split(" (")[0]
        for key in KEYS:
            os.environ.pop(key, None)
        parts = []
        for name, _ in VARIANTS:
            us = sorted(res[name])[len(res[name]) // 2]
            parts.append("%s %.1f (%.0f TF, %s)" % (name, us, fl / us / 1e6, kern[name]))
        print("wgrad %dx%d %d->%d k%d: " % (H, W, cin, cout, k) + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
