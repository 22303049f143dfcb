#!/bin/bash
# fused stem pool/BN backward: tests, then a same-box A/B against the two-launch form
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nnops.py tests/test_gpu_stem.py > gpurun_out/poolbn_pytest.log 2>&1 || { tail -30 gpurun_out/poolbn_pytest.log; exit 1; }
tail -2 gpurun_out/poolbn_pytest.log
bash tools/bench_ab.sh "" "CVL_DISPATCH=no_stem_pool_bwd_fuse"
