"""Times the stem kernels alone at the FCOS geometry (bs 16, 512x512): cvl_stem_conv7x7s2 and
cvl_stem_wgrad (+ its split reduction), mean of 20 launches after 3 warm-ups (HIP events).
usage: stem_probe.py [tag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    B, H = 16, 512
    img = (torch.rand((B, H, H, 3), device="cuda") * 2 - 1)
    wf = (torch.randn((64, 168), device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.zeros(64, device="cuda")
    z = torch.empty((B, 256, 256, 64), dtype=torch.bfloat16, device="cuda")
    st = nn.bn_acc(B, 64, "cuda")
    dz = (torch.randn((B, 256, 256, 64), device="cuda") * 0.01).to(torch.bfloat16)
    dw = torch.empty((192, 64), dtype=torch.float32, device="cuda")
    f = timed(lambda: nn.stem_conv7x7s2(img, wf, bias, z, st))
    w = timed(lambda: nn.stem_wgrad(img, dz, dw))
    print("%s stem fwd %.1f us, wgrad %.1f us" % (tag, f, w), flush=True)


if __name__ == "__main__":
    main()
