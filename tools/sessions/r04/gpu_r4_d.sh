#!/bin/bash
# Round-4 evidence: full GPU suite with the parity report, then the C2 profile set (bench, rocprof, 3 PMC passes).
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_r4.sh r4d2 "" "" p; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4d2 c2
