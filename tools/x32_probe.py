"""Tower conv (bench.measure_tower_conv, graph-free HIP events) under CVL_X_ABLATE settings."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CVL_LIB", os.path.join(ROOT, "ab", "libcvlite_measure.so"))  # tools/build_measure.sh
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
    for st in sys.argv[1:] or ["0"]:
        os.environ["CVL_X_ABLATE"] = st
        ms, fl, kn = bench.measure_tower_conv(net, 16, 512, 512, iters=20)
        print("ablate %-5s %.4f ms  %.1f TFLOP/s  %s" % (st, ms, fl / ms / 1e9, kn.split(" (")[0]), flush=True)
    os.environ.pop("CVL_X_ABLATE", None)


if __name__ == "__main__":
    main()
