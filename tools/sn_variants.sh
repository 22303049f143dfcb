#!/bin/bash
# measurement variants of conv_wgrad_sn.hip (-DCVL_SN_ABL=<bits>) into ab/libcvlite_sn<bits>.so
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
csrc=$root/cv-lite-object-detection_amd/csrc
make -s -C "$csrc" -j8 >/dev/null
objs=$(ls "$csrc"/build/*.o | grep -v conv_wgrad_sn.o)
for b in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast -DCVL_SN_ABL=$b -c "$csrc/conv_wgrad_sn.hip" -o /tmp/sn_$b.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/ab/libcvlite_sn$b.so" $objs /tmp/sn_$b.o
done
