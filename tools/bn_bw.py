"""Bandwidth probe of the BN elementwise kernels (bn_apply, bn_backward_relu_sums, bn_backward) at
the ResNet-50 stage shapes, against a torch copy of the same bytes: python tools/bn_bw.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cv-lite-object-detection_amd"))
from cvlite import ops_nn as nn  # noqa: E402

BF = torch.bfloat16
dev = "cuda"


def timeit(fn, reps=20):
    """us per launch: reps launches captured into a HIP graph and replayed (no host cost in the time)"""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3      # us


shapes = [(16, 16384, 256), (16, 16384, 64), (16, 4096, 512), (16, 4096, 128), (16, 1024, 1024), (16, 65536, 64),
          (16, 256, 2048)]
if os.environ.get("BNBW_SHAPES"):
    shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["BNBW_SHAPES"].split(",")]
for B, HW, C in shapes:
    n = B * HW * C
    z = torch.randn(n, device=dev).to(BF)
    r = torch.randn(n, device=dev).to(BF)
    dy = torch.randn(n, device=dev).to(BF)
    y = torch.empty(n, device=dev, dtype=BF)
    dz = torch.empty(n, device=dev, dtype=BF)
    mr = torch.stack([torch.zeros(B * C, device=dev), torch.ones(B * C, device=dev)], 1).contiguous()
    ga = torch.ones(C, device=dev)
    be = torch.zeros(C, device=dev)
    sums = nn.bn_acc(B, C, dev)
    dga = torch.zeros(C, device=dev)
    dbe = torch.zeros(C, device=dev)
    t_cp = timeit(lambda: y.copy_(z))
    t_add = timeit(lambda: torch.add(z, r, out=y))
    t_a = timeit(lambda: nn.bn_apply(z, mr, ga, be, None, y, B, HW, C, 1))
    t_ar = timeit(lambda: nn.bn_apply(z, mr, ga, be, r, y, B, HW, C, 1))
    t_p1 = timeit(lambda: nn.bn_backward_relu_sums(dy, z, mr, ga, be, sums, dz, dga, dbe, B, HW, C))
    t_full = timeit(lambda: nn.bn_backward(dy, y, z, mr, ga, dz, None, dga, dbe, B, HW, C))
    mb = n * 2 / 1e6
    print(f"B{B} HW{HW} C{C} ({mb:.0f} MB/tensor): copy {t_cp:.1f}us {2*mb/t_cp:.2f}TB/s | add {t_add:.1f}us {3*mb/t_add:.2f} | apply {t_a:.1f}us "
          f"{2*mb/t_a:.2f} | apply+res {t_ar:.1f}us {3*mb/t_ar:.2f} | bwd pass1(relu,sums) {t_p1:.1f}us "
          f"{3*mb/t_p1:.2f} | bwd full(y mask) {t_full:.1f}us {7*mb/t_full:.2f}", flush=True)
