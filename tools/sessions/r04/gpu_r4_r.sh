#!/bin/bash
# Round-4 session R: whole GPU suite + smoke on the final tree.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4r/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -1 gpurun_out/r4r/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4.sh r4r "" "" p
