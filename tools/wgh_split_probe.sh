#!/bin/bash
# Kernel-only time of the 3x3 weight-gradient (WH) launches under forced workgroup targets
# (measurement library, CVL_WGH_WGS = workgroups the planner aims at): fixed vs per-step cost.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in ${*:-256 128 64}; do
  CVL_WGH_WGS=$w WGX_CHILD=0 CVL_LIB=ab/libcvlite_measure.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/r06p_wgh$w -o p -- python3 tools/wgx_probe.py > gpurun_out/r06p_wgh$w.txt 2>&1 || exit 1
done
python3 - "$@" <<'PY'
import collections, csv, sys
for w in (sys.argv[1:] or ["256", "128", "64"]):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open("gpurun_out/r06p_wgh%s/p_kernel_trace.csv" % w)):
        if "wgrad_h_kernel" in r["Kernel_Name"] or "reduce_batch" in r["Kernel_Name"]:
            k = ("WH" if "wgrad_h" in r["Kernel_Name"] else "red", int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
            agg[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print("WGS %s: %s" % (w, "; ".join("%s %d WGs n=%d med %.1f" % (k[0], k[1], len(v), sorted(v)[len(v) // 2])
                                       for k, v in sorted(agg.items()) if len(v) >= 20)))
PY
