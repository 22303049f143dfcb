"""Checksums of the H64 backbone 3x3 forwards (conv2_x 64->64 @ 128^2 incl. its BN statistics, conv4_x
256->256 @ 32^2) at bs 16 from fixed inputs, for bit-identity A/Bs of H64 variants: run once per
variant (env knob / build) and compare the lines (round 4: the register-staged halo experiment)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    net = FCOSNet(bench.NUM_CLASSES, device=torch.device("cuda", 0), seed=0)
    B, h, w = 16, 128, 128
    g = torch.Generator(device="cpu").manual_seed(7)
    for si, stage in enumerate(net.backbone.stages):
        if si > 0:
            h, w = h // 2, w // 2
        if si not in (0, 2):
            continue
        conv = stage[-1].c2.conv
        x = torch.randn((B, h, w, conv.cin), generator=g).to(torch.bfloat16).cuda()
        y = torch.zeros((B, h, w, conv.cout), dtype=torch.bfloat16, device="cuda")
        st = nn.bn_acc(B, conv.cout, "cuda")
        fd = conv.fwd_desc(B, [nn.seg(h, w, h, w, conv.wf, conv.bias_arg())], ld_dst=conv.cout)
        nn.conv_igemm(fd, x, y, st)
        torch.cuda.synchronize()
        hy = hashlib.sha1(y.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
        hs = hashlib.sha1(st.cpu().numpy().tobytes()).hexdigest()[:16]
        print("stage %d fwd: y %s stats %s (|y| sum %.6e)" % (si, hy, hs, y.float().abs().sum().item()))


if __name__ == "__main__":
    main()
