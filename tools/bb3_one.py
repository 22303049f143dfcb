"""Runs the 12 distinct backbone 3x3 launches of one FCOS step (ResNet-50 conv2_x..conv5_x `_2_conv`,
bs 16, 512x512: fwd with BN statistics, the fused-BN-sums data gradient, the weight gradient) N
times each, for rocprofv3 --pmc passes (tools/pmc_bb3.sh); prints one line per launch with its
kernel, grid and the HIP-event time.  usage: python tools/bb3_one.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    net = FCOSNet(bench.NUM_CLASSES, device=torch.device("cuda", 0), seed=0)
    r = bench.measure_backbone_3x3(net, 16, 512, 512, iters=iters, eager=True)
    for row in r["per_shape"]:
        print(row)
    print("backbone_3x3 frac", r["frac"], "ms/step", r["ms_per_step"])


if __name__ == "__main__":
    main()
