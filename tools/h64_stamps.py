"""In-kernel wall-clock stamps of the H64 kernel (CVL_X_ABLATE bit 256) on the backbone 3x3 forward
launches: per workgroup entry / set-up / prologue / main loop / exit times and placement."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite import ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
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
        st = nn.bn_acc(B, conv.cout, "cuda")
        fd = conv.fwd_desc(B, [nn.seg(h, w, h, w, conv.wf, conv.bias_arg())], ld_dst=conv.cout)
        for ab in (256 | extra,):
            os.environ["CVL_X_ABLATE"] = str(ab)
            for _ in range(3):
                nn.conv_igemm(fd, x, y, st)
            torch.cuda.synchronize()
            s = y.view(torch.int64).view(-1, 8).cpu()
            n = (s[:, 0] > 0).sum().item()
            s = s[:n].double()
            t0 = s[:, 0].min()
            ent, setup, pro, loop, ex = [(s[:, k] - (s[:, k - 1] if k else t0)) / 100.0 for k in range(5)]
            span = (s[:, 4].max() - t0) / 100.0
            print("stage %d C %d ablate %d: %d WGs, span %.1f us | per WG: setup %.2f prologue %.2f loop %.2f "
                  "exit %.2f us (medians); entry times: first %.1f median %.1f last %.1f; XCC %s" % (
                      si, C, ab, n, span, setup.median(), pro.median(), loop.median(), ex.median(),
                      0.0, ent.median(), ent.max(), sorted(set(int(v) for v in s[:, 6].tolist()))[:8]))
            order = torch.argsort(s[:, 0])
            ent_sorted = ((s[order, 0] - t0) / 100.0).tolist()
            print("   entry us of WG #0,255,256,511,512,767,768,1023:",
                  [round(ent_sorted[i], 1) for i in (0, 255, 256, 511, 512, 767, 768, 1023) if i < n])
    os.environ.pop("CVL_X_ABLATE", None)


if __name__ == "__main__":
    main()
