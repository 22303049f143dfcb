#!/bin/bash
# One-GPU cost of the data-parallel step form: the default bench line vs the same
# step with the all-reduce path live on a one-rank RCCL group (CVL_DISPATCH=dp_force_sync: the
# fwd+bwd graph captured in hook-split segments, async all-reduces between segment replays, the
# update queued behind them).  Same box, alternating, 2 rounds; the force-sync lines carry the
# per-group enqueue points (dist.grad_allreduce); a third arm keeps the segmented graphs but issues
# no collective (CVL_DISPATCH=dp_segments_only).  Output: gpurun_out/dp_*.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 30 --runs 3 --no-cpu-baseline > gpurun_out/dp_off_$r.json 2> gpurun_out/dp_off_$r.err || exit 1
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + r)) RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 CVL_DISPATCH=dp_force_sync \
    timeout -k 10 150 python -u bench.py --steps 30 --runs 3 --no-cpu-baseline > gpurun_out/dp_on_$r.json 2> gpurun_out/dp_on_$r.err || exit 1
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29610 + r)) RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 CVL_DISPATCH=dp_force_sync,dp_segments_only \
    timeout -k 10 150 python -u bench.py --steps 30 --runs 3 --no-cpu-baseline > gpurun_out/dp_seg_$r.json 2> gpurun_out/dp_seg_$r.err || exit 1
  python3 - "$r" <<'EOF'
import json, sys
r = sys.argv[1]
off, on, seg = (json.loads(open("gpurun_out/dp_%s_%s.json" % (k, r)).read().strip().splitlines()[-1])
                for k in ("off", "on", "seg"))
print("round %s: default %.1f img/s (%.3f ms)  force-sync %.1f img/s (%.3f ms)  overhead %.2f %%  "
      "(segmented graphs alone, no collective: %.3f ms, %.2f %%)"
      % (r, off["value"], off["ms_per_step"], on["value"], on["ms_per_step"],
         100.0 * (on["ms_per_step"] / off["ms_per_step"] - 1.0), seg["ms_per_step"],
         100.0 * (seg["ms_per_step"] / off["ms_per_step"] - 1.0)))
ga = on["dist"]["grad_allreduce"]
if ga.get("live"):
    print("  traced step %.3f ms; group: buckets MB, ready ms, all-reduce done ms" % ga["traced_step_ms"])
    for g in ga["groups"]:
        print("  %-14s %-22s %8.3f %8.3f" % (g["group"], g["bucket_mb"], g["ready_ms"], g["allreduce_done_ms"]))
EOF
done
