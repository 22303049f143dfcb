"""Replays the FCOS cls-head weight gradient (3x3 256 -> 20 over the five levels at 512 / bs 16, one
grouped call, group = level) for a kernel trace: rocprofv3 --kernel-trace --stats -- python3 tools/sn_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn  # noqa: E402

BF = torch.bfloat16
B, C, ld = 16, 256, 32
n_store = int(os.environ.get("SN_NSTORE", "20"))
shapes = [(64, 64), (32, 32), (16, 16), (8, 8), (4, 4)]
off, o = [], 0
for h, w in shapes:
    off.append(o)
    o += h * w
P = o
x = torch.randn(B * P, C, device="cuda").to(BF)
dy = torch.randn(B * P, ld, device="cuda").to(BF)
wf = [torch.empty((32, 9 * C), dtype=BF, device="cuda") for _ in shapes]
segs = [nn.seg(h, w, h, w, wf[l], None, src_base=B * off[l], src_img=h * w, dst_base=off[l], dst_img=P)
        for l, (h, w) in enumerate(shapes)]
d = nn.make_desc(nn.FWD, B, C, 3, 3, 1, 1, 1, 32, n_store, ld, segs)
dws = [torch.zeros((3, 3, C, n_store), device="cuda") for _ in shapes]
for _ in range(int(os.environ.get("SN_REPS", "50"))):
    nn.conv_wgrad_grouped(d, x, dy, dws)
torch.cuda.synchronize()
print("ok")
