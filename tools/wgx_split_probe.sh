#!/bin/bash
# Kernel-only time (rocprofv3 kernel trace) of the weight-gradient launches under forced split counts
# (measurement library, CVL_WGX_SPLITS): what one workgroup's fixed costs amortise to with longer chunks.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in ${*:-16 8 4 2 1}; do
  CVL_WGX_SPLITS=$s WGX_CHILD=0 CVL_LIB=ab/libcvlite_measure.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/r06i_split$s -o p -- python3 tools/wgx_probe.py > gpurun_out/r06i_split$s.txt 2>&1 || exit 1
done
