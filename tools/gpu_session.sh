#!/bin/bash
# One GPU call, several measurements: tools/gpu_session.sh <tag> [steps...]
# steps: tests bench table wgx prof ceiling (default: all; limits sum to 1080 s).  Each step has its own time limit; a
# fault / abort / time-out (exit 124, 134, 137, 139) ends the session there.  Output: gpurun_out/<tag>_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
steps=${*:-tests bench table wgx prof ceiling}
run() {   # run <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  echo "== $* ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local st=$?
  echo "   exit $st"
  case $st in 124|134|137|139) echo "   fault/timeout: stopping"; exit $st ;; esac
  return 0
}
for s in $steps; do
  case $s in
    tests)   run 540 gpurun_out/${tag}_pytest.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
             tail -4 gpurun_out/${tag}_pytest.log ;;
    bench)   run 150 gpurun_out/${tag}_bench.err bash -c "python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/${tag}_bench.json"
             tail -c 300 gpurun_out/${tag}_bench.json; echo ;;
    benchs)  run 150 gpurun_out/${tag}_benchs.err bash -c "CVL_DISPATCH=no_sc_bn_fuse python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/${tag}_benchs.json"
             tail -c 200 gpurun_out/${tag}_benchs.json; echo ;;
    benchx)  run 150 gpurun_out/${tag}_benchx.err bash -c "CVL_BN_EXACT=1 python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/${tag}_benchx.json"
             tail -c 200 gpurun_out/${tag}_benchx.json; echo ;;
    table)   run 120 gpurun_out/${tag}_table.log python -u tools/conv_table.py --out gpurun_out/${tag}_conv_table.md
             head -4 gpurun_out/${tag}_conv_table.md ;;
    wgx)     run 90 gpurun_out/${tag}_wgx.md python -u tools/wgx_stamps.py ;;
    prof)    run 150 gpurun_out/${tag}_prof.log rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${tag}_prof -o p -- python3 bench.py --steps 10 --warmup 5 --runs 1 --no-cpu-baseline ;;
    hash)    run 120 gpurun_out/${tag}_hash.txt python -u tools/step_hash.py; cat gpurun_out/${tag}_hash.txt ;;
    dp)      run 700 gpurun_out/${tag}_dp.txt bash tools/dp_overhead.sh; cat gpurun_out/${tag}_dp.txt ;;
    ceiling) run 30 gpurun_out/${tag}_ceiling.json ./tools/mfma_ceiling; cat gpurun_out/${tag}_ceiling.json ;;
    rowdma)  run 60 gpurun_out/${tag}_rowdma.txt ./tools/ubench_rowdma; cat gpurun_out/${tag}_rowdma.txt ;;
    pprobe)  run 90 gpurun_out/${tag}_pprobe.md python -u tools/p_probe.py; cat gpurun_out/${tag}_pprobe.md ;;
    pstamps) run 90 gpurun_out/${tag}_pstamps.txt python -u tools/p_stamps.py; cat gpurun_out/${tag}_pstamps.txt ;;
    hstamps) run 90 gpurun_out/${tag}_hstamps.md python -u tools/h64_stamps.py; cat gpurun_out/${tag}_hstamps.md ;;
    stem)    run 200 gpurun_out/${tag}_stem.log python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_bn_acc.py -q --timeout 150 --timeout-method thread
             tail -3 gpurun_out/${tag}_stem.log ;;
  esac
done
