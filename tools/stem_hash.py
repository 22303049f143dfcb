"""SHA-1 prefixes of the stem forward's z and BN statistics at the FCOS geometry (bs 16, 512x512) from a
fixed seed: compare two builds (CVL_LIB) for bit-identity.  usage: stem_hash.py"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn  # noqa: E402

g = torch.Generator(device="cpu").manual_seed(11)
B, H = 16, 512
img = (torch.rand((B, H, H, 3), generator=g) * 2 - 1).cuda()
w = (torch.randn((7, 7, 3, 64), generator=g) * 0.1)
wf = torch.zeros((64, 7, 24), dtype=torch.float32)
wf[:, :, :21] = w.permute(3, 0, 1, 2).reshape(64, 7, 21)
wf = wf.reshape(64, 168).to(torch.bfloat16).cuda()
bias = (torch.randn(64, generator=g) * 0.1).cuda()
z = torch.empty((B, 256, 256, 64), dtype=torch.bfloat16, device="cuda")
st = nn.bn_acc(B, 64, "cuda")
nn.stem_conv7x7s2(img, wf, bias, z, st)
torch.cuda.synchronize()
h = lambda t: hashlib.sha1(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
print("z", h(z), "stats", h(st))
