#!/bin/bash
# shortcut BN first pass fused into the residual unit's second pass: tests + A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_launch_parity.py tests/test_gpu_fcos_step.py tests/test_gpu_model.py tests/test_gpu_configs0.py tests/test_gpu_dp.py > gpurun_out/sc_pytest.log 2>&1 || { tail -40 gpurun_out/sc_pytest.log; exit 1; }
tail -1 gpurun_out/sc_pytest.log
grep -h "res_sums_sc\|bn_backward_sums " gpurun_out/launch_parity_fcos_512_bs16.txt | head -8
head -1 gpurun_out/launch_parity_fcos_512_bs16.txt
bash tools/bench_ab.sh "" "CVL_DISPATCH=no_sc_bnsum"
grep -c "bn_backward_sc " gpurun_out/launch_parity_fcos_512_bs16.txt
