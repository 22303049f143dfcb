#!/bin/bash
# RCCL path on a 1-GPU box: the one-rank nccl test, then bench.py under torchrun with the gradient
# all-reduce forced on (segmented graphs + async RCCL between replays) vs the plain N=1 bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/nccl_pytest.log 2>&1 || { tail -40 gpurun_out/nccl_pytest.log; exit 1; }
tail -4 gpurun_out/nccl_pytest.log
CVL_DP_FORCE_SYNC=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nccl_bench.json 2> gpurun_out/nccl_bench.err || { tail -30 gpurun_out/nccl_bench.err; exit 1; }
cat gpurun_out/nccl_bench.json
