cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 120 python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/h9_a$r.json 2>gpurun_out/h9_a$r.err || exit 1
CVL_WGX_SR=32 timeout -k 10 120 python -u bench.py --steps 30 --runs 1 --no-cpu-baseline > gpurun_out/h9_b$r.json 2>gpurun_out/h9_b$r.err || exit 1
done
