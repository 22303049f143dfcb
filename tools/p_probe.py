"""Time single 1x1 conv launches (graph replay) under environment settings: p_probe.py "" "X=1" ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn, _lib  # noqa: E402

CASES = [(16, 128, 64, 256, 1, True), (16, 128, 256, 64, 1, True), (16, 64, 128, 512, 1, True),
         (16, 32, 256, 1024, 1, True), (16, 32, 1024, 256, 1, True), (16, 16, 2048, 512, 1, True),
         (16, 16, 512, 2048, 1, True), (16, 16, 2048, 256, 1, False)]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream()
    e0.record(s)
    g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    settings = sys.argv[1:] or [""]
    L = _lib.load()
    gen = torch.Generator(device="cpu").manual_seed(0)
    rows = []
    for (B, H, Cin, Cout, st, stats) in CASES:
        x = torch.randn((B, H, H, Cin), generator=gen).to(torch.bfloat16).cuda()
        w = (torch.randn((Cout, Cin), generator=gen) * Cin ** -0.5).to(torch.bfloat16).cuda()
        y = torch.empty((B, H, H, Cout), dtype=torch.bfloat16, device="cuda")
        sts = nn.bn_acc(B, Cout, "cuda") if stats else None
        d = nn.make_desc(nn.FWD, B, Cin, 1, 1, 1, 0, 0, Cout, Cout, Cout, [nn.seg(H, H, H, H, w, None)])
        row = ["fwd 1x1 %d->%d @ %dx%d" % (Cin, Cout, H, H)]
        mb = (x.numel() + y.numel()) * 2 / 1e6
        for stt in settings:
            kv = [t.split("=", 1) for t in stt.split()]
            for k, v in kv:
                os.environ[k] = v
            us = timed(lambda: nn.conv_igemm(d, x, y, sts))
            kn = L.cvl_conv_kernel_name(L.cvl_conv_igemm_last_kernel()).decode().split(" ")[0]
            for k, _ in kv:
                del os.environ[k]
            row.append("%.1f us %.0f GB/s %s" % (us, mb / us * 1e3, kn[:14]))
        rows.append(row)
    print("| launch | " + " | ".join(repr(s) for s in settings) + " |")
    for r in rows:
        print("| " + " | ".join(r) + " |")


if __name__ == "__main__":
    main()
