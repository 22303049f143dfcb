#!/bin/bash
# Kernel-only times (rocprofv3 kernel trace) of the weight-gradient launches of tools/wgx_probe.py for
# ablation variant libraries ab/libcvlite_wgx<bits>.so (tools/wgx_probe.sh): tools/wgx_var_prof.sh <tag> bits...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
for b in "$@"; do
  WGX_CHILD=$b CVL_LIB=ab/libcvlite_wgx$b.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/${tag}_v$b -o p -- python3 tools/wgx_probe.py > gpurun_out/${tag}_v$b.txt 2>&1 || exit 1
done
python3 tools/wgx_trace_summary.py gpurun_out/${tag}_v "$@"
