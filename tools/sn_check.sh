#!/bin/bash
# small-N head weight gradient: parity tests, then the conv table (gpurun_out/conv_table_<tag>.md)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py -k "small_n" > gpurun_out/sn_pytest.log 2>&1 || { tail -30 gpurun_out/sn_pytest.log; exit 1; }
tail -2 gpurun_out/sn_pytest.log
timeout -k 10 300 python3 tools/conv_table.py --out gpurun_out/conv_table_${1:-sn}.md > gpurun_out/conv_table_${1:-sn}.log 2>&1 || exit 1
grep -E "Total|wgrad 3x3 256->(20|5) " gpurun_out/conv_table_${1:-sn}.md
