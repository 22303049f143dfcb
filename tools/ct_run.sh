#!/bin/bash
# conv table of the FCOS step (configs[1]) into gpurun_out/conv_table_<tag>.md
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/conv_table.py --out gpurun_out/conv_table_${1:-x}.md > gpurun_out/conv_table_${1:-x}.log 2>&1
