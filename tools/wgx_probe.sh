#!/bin/bash
# Build-side half of the un-instrumented weight-gradient ablation probe: one product library per
# ablation value with conv_wgrad_x.hip compiled -DCVL_WGX_ABL=<bits> (1 no fragment reads, 2 no memory
# traffic, 16 no MFMAs, 32 no DMA instructions) into ab/libcvlite_wgx<bits>.so.  usage: wgx_probe.sh bits...
# GPU side: python tools/wgx_probe.py <bits...> (each variant in its own process).
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
csrc=$root/cv-lite-object-detection_amd/csrc
make -s -C "$csrc" -j8 >/dev/null
mkdir -p "$root/ab"
objs=$(ls "$csrc"/build/*.o | grep -v conv_wgrad_x.o)
for b in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast -DCVL_WGX_ABL=$b -c "$csrc/conv_wgrad_x.hip" -o /tmp/wgx_$b.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/ab/libcvlite_wgx$b.so" $objs /tmp/wgx_$b.o
  echo "built ab/libcvlite_wgx$b.so"
done
