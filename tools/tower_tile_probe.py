"""Probe: tower 3x3 conv fwd at batch B (B=32 stands in for a fused cls+reg tower launch, twice
the rows of one bs=16 tower conv) with the current tile choice; run under different
CVL_CONV_L256_MIN_TILES to compare the 256x256 and 128-wide tiles.  usage: tower_tile_probe.py B"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
net = FCOSNet(bench.NUM_CLASSES, device="cuda", seed=0)
ms, fl = bench.measure_tower_conv(net, B, 512, 512, iters=30)
print("B=%d L256_MIN=%s tower conv %.4f ms/launch, %.1f TFLOP/s" % (
    B, os.environ.get("CVL_CONV_L256_MIN_TILES", "512"), ms, fl / ms / 1e9), flush=True)
