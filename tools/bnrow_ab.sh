cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nnops.py tests/test_gpu_bn_acc.py tests/test_gpu_fcos_step.py tests/test_gpu_hourglass.py tests/test_gpu_mobilenet.py > gpurun_out/bnrow_pytest.log 2>&1 && tail -2 gpurun_out/bnrow_pytest.log &&
timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_new.txt 2>&1 &&
CVL_LIB=ab/libcvlite_base.so timeout -k 10 200 python3 tools/step_hash.py > gpurun_out/h_base.txt 2>&1 &&
(diff gpurun_out/h_new.txt gpurun_out/h_base.txt && echo HASH_SAME || echo HASH_DIFF) &&
BNBW_SHAPES=16x256x512,16x256x2048,16x1024x256,16x1024x1024,16x4096x128,16x16384x64 bash tools/bn_bw.sh CVL_LIB=ab/libcvlite_base.so &&
bash tools/bench_ab.sh "" "CVL_LIB=ab/libcvlite_base.so"
