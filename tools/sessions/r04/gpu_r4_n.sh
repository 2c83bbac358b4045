#!/bin/bash
# Round-4 session N: the whole GPU suite on the final tree, smoke, C2 bench line.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4n2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n2/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -1 gpurun_out/r4n2/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4.sh r4n2 "" "" pb
