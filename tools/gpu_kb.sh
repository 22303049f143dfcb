set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/kbench.py > gpurun_out/kb_def.log 2>&1 || { tail -20 gpurun_out/kb_def.log; exit 1; }
CVL_CONV_NO_L=1 timeout -k 10 120 python -u tools/kbench.py > gpurun_out/kb_nol.log 2>&1 || { tail -20 gpurun_out/kb_nol.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s4c_bench.json 2> gpurun_out/s4c_bench.err || { tail -30 gpurun_out/s4c_bench.err; exit 1; }
cut -c1-200 gpurun_out/s4c_bench.json
