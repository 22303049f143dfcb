"""A/B of tower-conv variants by environment (graph-free events, bench.measure_tower_conv, repeated)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    settings = sys.argv[1:] or [""]
    for rep in range(3):
        for st in settings:
            kv = [t.split("=", 1) for t in st.split()]
            for k, v in kv:
                os.environ[k] = v
            ms, fl, kn = bench.measure_tower_conv(net, 16, 512, 512, iters=30)
            for k, _ in kv:
                del os.environ[k]
            print("rep %d %-30r %.4f ms %.1f TFLOP/s" % (rep, st, ms, fl / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
