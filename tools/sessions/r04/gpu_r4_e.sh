#!/bin/bash
# Round-4 session E: smoke(), conv A/B of 64-row tiles (3 workgroups per CU), the C4 profile set.
set -u
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r4e_smoke.log 2>&1; rc=$?
tail -2 gpurun_out/r4e_smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_conv_ab.sh r4e_conv conv_bm=64; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4e c4
