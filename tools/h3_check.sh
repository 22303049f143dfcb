#!/bin/bash
# H64 three-stage 32-wide tiles: conv tests, launch parity, conv table rows, same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv_h.py tests/test_gpu_conv.py tests/test_gpu_conv_production.py tests/test_gpu_launch_parity.py > gpurun_out/h3_pytest.log 2>&1 || { tail -40 gpurun_out/h3_pytest.log; exit 1; }
tail -1 gpurun_out/h3_pytest.log
head -1 gpurun_out/launch_parity_fcos_512_bs16.txt
for f in "" "CVL_DISPATCH=h_no_3stage"; do env $f timeout -k 10 300 python3 tools/conv_table.py --out gpurun_out/ct_h3.md > /dev/null 2>&1 || exit 1; echo "== $f"; grep -E "Total|256->(20|5) |3x3 512->512" gpurun_out/ct_h3.md; done
bash tools/bench_ab.sh "" "CVL_DISPATCH=h_no_3stage"
