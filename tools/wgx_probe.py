"""Weight-gradient launches of one FCOS step (512x512 bs 16) replayed alone and timed by HIP events
(no in-kernel stamps: the loop is un-instrumented) for ablation variants of the kernel built by
tools/wgx_probe.sh into ab/libcvlite_wgx<bits>.so (1 no fragment reads, 2 DMA out of range: no
traffic, 16 no MFMAs, 32 no DMA instructions).  usage: wgx_probe.py bits...  -- one child process per
variant (the library is chosen at import); each time includes the launch's split reduction."""
import subprocess
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from conv_table import desc_key, describe  # noqa: E402
from cvlite import _lib, ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402
from cvlite.train_fcos import FCOSTrainer, synthetic_batch  # noqa: E402

KEEP = ("1x1 1024->256 @ 32x32", "1x1 64->256 @ 128x128", "3x3 256->256 @ 64x64 +9", "3x3 256->256 @ 32x32",
        "3x3 64->64 @ 128x128")


def one(bits):
    B, H = 16, 512
    net = FCOSNet(20, device=torch.device("cuda"), seed=0)
    tr = FCOSTrainer(net, B, (H, H), use_graph=False)
    tr.load_batch(*synthetic_batch(B, H, H, 20, seed=1234, device="cuda"))
    tr.step()
    torch.cuda.synchronize()
    calls = collections.OrderedDict()
    orig = (nn.conv_wgrad, nn.conv_wgrad_grouped)

    def wgrad(desc, x, dy, dw, beta=0.0):
        calls.setdefault(desc_key("wgrad", desc), (lambda: orig[0](desc, x, dy, dw, beta), desc, 1))
        return orig[0](desc, x, dy, dw, beta)

    def wgrad_g(desc, x, dy, dws, beta=0.0):
        calls.setdefault(desc_key("wgrad_g", desc), (lambda: orig[1](desc, x, dy, dws, beta), desc, len(dws)))
        return orig[1](desc, x, dy, dws, beta)

    nn.conv_wgrad, nn.conv_wgrad_grouped = wgrad, wgrad_g
    tr.step()
    torch.cuda.synchronize()
    nn.conv_wgrad, nn.conv_wgrad_grouped = orig
    sel = [(describe("wgrad", d, ng), r) for k, (r, d, ng) in calls.items()]
    sel = [(n, r) for n, r in sel if any(s in n for s in KEEP)]
    out = []
    for name, replay in sel:
        row = []
        for a in [bits]:
            for _ in range(3):
                replay()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()            # 20 launches captured: no host cost in the timing
            with torch.cuda.graph(g):
                for _ in range(20):
                    replay()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            row.append(e0.elapsed_time(e1) * 1000 / 20)
        out.append((name, row[0]))
    return out


def main():
    if os.environ.get("WGX_CHILD"):
        for name, us in one(os.environ["WGX_CHILD"]):
            print("%s\t%.2f" % (name, us), flush=True)
        return
    bits = sys.argv[1:] or ["0"]
    cols = {}
    for b in bits:
        env = dict(os.environ, WGX_CHILD=b, CVL_LIB=os.path.join(ROOT, "ab", "libcvlite_wgx%s.so" % b))
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                           timeout=150)
        if r.returncode:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
        cols[b] = dict(line.split("\t") for line in r.stdout.strip().splitlines())
    names = list(cols[bits[0]])
    print("| launch | " + " | ".join("ablate %s us" % b for b in bits) + " |")
    print("|---|" + "---|" * len(bits))
    for n in names:
        print("| %s | %s |" % (n, " | ".join(cols[b].get(n, "-") for b in bits)))


if __name__ == "__main__":
    main()
