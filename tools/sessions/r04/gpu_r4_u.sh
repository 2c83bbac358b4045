#!/bin/bash
# Round-4 session U: final tree -- whole GPU suite, smoke, C2 profile set.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4u
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -1 gpurun_out/r4u/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4.sh r4u "" "" p; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4u c2
