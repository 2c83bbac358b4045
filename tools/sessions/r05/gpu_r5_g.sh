#!/bin/bash
# Round-5 session G: the full GPU suite + smoke + bench (tools/gpu_check.sh),
# then the C2 rocprof kernel-trace + PMC profile of the same build.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_check.sh r5g_chk || exit $?
bash tools/gpu_prof.sh r5g_prof c2 || exit $?
