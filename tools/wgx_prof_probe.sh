cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 0 241; do
  WGX_CHILD=$b CVL_LIB=ab/libcvlite_wgx$b.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r06h_prof$b -o p -- python3 tools/wgx_probe.py > gpurun_out/r06h_$b.txt 2>&1 || exit 1
done
ls -R gpurun_out/r06h_prof0 | head
