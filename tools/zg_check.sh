#!/bin/bash
# zero_gaps rewrite: step hash vs the HEAD build, conv tests, same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_new.txt 2>&1 &&
CVL_LIB=ab/libcvlite_base.so timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_base.txt 2>&1 &&
(diff gpurun_out/h_new.txt gpurun_out/h_base.txt > /dev/null && echo HASH_SAME || echo HASH_DIFF) &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_launch_parity.py > gpurun_out/zg_pytest.log 2>&1; tail -1 gpurun_out/zg_pytest.log
bash tools/bench_ab.sh "" "CVL_LIB=ab/libcvlite_base.so"
