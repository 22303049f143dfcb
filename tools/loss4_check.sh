#!/bin/bash
# four-lanes-per-cell FCOS loss: bit-identity tests + step tests, kernel times, same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_targets_loss.py tests/test_gpu_fcos_step.py tests/test_gpu_fullsize.py tests/test_gpu_fcos_center.py > gpurun_out/l4_pytest.log 2>&1 || { tail -30 gpurun_out/l4_pytest.log; exit 1; }
tail -1 gpurun_out/l4_pytest.log
timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_new.txt 2>&1 &&
CVL_DISPATCH=loss_lds1 timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_base.txt 2>&1 &&
(diff gpurun_out/h_new.txt gpurun_out/h_base.txt > /dev/null && echo HASH_SAME || echo HASH_DIFF) &&
bash tools/bench_ab.sh "" "CVL_DISPATCH=loss_lds1"
