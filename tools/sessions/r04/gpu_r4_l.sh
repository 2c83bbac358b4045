#!/bin/bash
# Round-4 session L: final C2 profile set (bench line, rocprof kernel trace, PMC passes) + smoke.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4l
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -2 gpurun_out/r4l/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4l c2
