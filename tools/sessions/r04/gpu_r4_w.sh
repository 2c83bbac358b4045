#!/bin/bash
# Round-4 session W: final tree -- whole GPU suite, smoke, C2 + C4 + C5 profile sets.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4w
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4w/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -1 gpurun_out/r4w/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4.sh r4w "" "" p; rc=$?
[ $rc -eq 0 ] || exit $rc
grep -q " failed" gpurun_out/r4w/pytest_gpu.log && exit 1
bash tools/gpu_prof.sh r4w c2 c4 c5
