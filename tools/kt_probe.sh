cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/kt_a -o kt -- python3 tools/bb3_probe.py "" CVL_X_ABLATE=15 > gpurun_out/kt_a.log 2>&1 || { tail gpurun_out/kt_a.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
p = glob.glob('gpurun_out/kt_a/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(p)))
seq = [(r['Kernel_Name'].replace('(anonymous namespace)::','')[:60], r['Grid_Size_X'], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000.0, int(r['Start_Timestamp'])) for r in rows]
seq.sort(key=lambda x: x[3])
d = collections.OrderedDict()
for n, g, t, s in seq:
    if 'conv' in n or 'wgrad' in n or 'finish' in n:
        d.setdefault((n, g), []).append(t)
for k, v in d.items():
    print(len(v), k, ' '.join('%.1f' % x for x in v[:8]), '...', ' '.join('%.1f' % x for x in v[-8:]))
PY
