"""Per-kernel timing of the conv kernels on the FCOS-R50 512x512 bs=16 shapes (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn  # noqa: E402
from cvlite.layers import Conv, ParamStore, same_pad  # noqa: E402

BF = torch.bfloat16
B = 16
# (name, H, W, Cin, Cout, k, stride)
SHAPES = [
    ("conv2 3x3 64", 128, 128, 64, 64, 3, 1),
    ("conv2 1x1 64->256", 128, 128, 64, 256, 1, 1),
    ("conv2 1x1 256->64", 128, 128, 256, 64, 1, 1),
    ("conv3 3x3 128", 64, 64, 128, 128, 3, 1),
    ("conv3 1x1 s2 256->512", 128, 128, 256, 512, 1, 2),
    ("conv4 3x3 256", 32, 32, 256, 256, 3, 1),
    ("conv4 1x1 1024->256", 32, 32, 1024, 256, 1, 1),
    ("conv5 3x3 512", 16, 16, 512, 512, 3, 1),
    ("conv5 1x1 512->2048", 16, 16, 512, 2048, 1, 1),
    ("c6 3x3 s2 2048->256", 16, 16, 2048, 256, 3, 2),
    ("P3 3x3 256", 64, 64, 256, 256, 3, 1),
]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    st = ParamStore()
    convs = [Conv(st, "c%d" % i, k, cin, cout, stride=s) for i, (_, H, W, cin, cout, k, s) in enumerate(SHAPES)]
    st.finalize("cuda", 0)
    for c in convs:
        c.pack()
    tot = {"fwd": 0, "dgrad": 0, "wgrad": 0}
    for (name, H, W, cin, cout, k, s), c in zip(SHAPES, convs):
        Ho, Wo, _, _ = c.out_hw(H, W)
        x = torch.randn((B, H, W, cin), device="cuda").to(BF)
        dy = torch.randn((B, Ho, Wo, cout), device="cuda").to(BF)
        out = torch.empty((B, Ho, Wo, cout), dtype=BF, device="cuda")
        dx = torch.empty((B, H, W, cin), dtype=BF, device="cuda")
        fl = 2.0 * B * Ho * Wo * cout * k * k * cin
        r = []
        for mode, fn in (("fwd", lambda: c.fwd(x, B, H, W, out=out)),
                         ("dgrad", lambda: c.dgrad(dy, B, H, W, out=dx)),
                         ("wgrad", lambda: c.wgrad(x, dy, B, H, W, bias=False))):
            ms = timeit(fn)
            tot[mode] += ms
            r.append("%s %7.3f ms %6.0f TF/s" % (mode, ms, fl / ms / 1e9))
        print("%-24s %s" % (name, " | ".join(r)), flush=True)
    print("totals (ms):", {k: round(v, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
