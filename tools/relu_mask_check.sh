#!/bin/bash
# masked head data gradient: tests (unit, launch parity, FCOS step), then a same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv.py::test_conv_igemm_relu_mask_matches_dgrad_then_relu tests/test_gpu_launch_parity.py tests/test_gpu_fcos_step.py > gpurun_out/rm_pytest.log 2>&1 || { tail -30 gpurun_out/rm_pytest.log; exit 1; }
tail -1 gpurun_out/rm_pytest.log
bash tools/bench_ab.sh "" "CVL_DISPATCH=no_top_relu_fuse"
