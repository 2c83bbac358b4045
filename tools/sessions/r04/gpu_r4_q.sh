#!/bin/bash
# Round-4 session Q: final C4 and C5 profile sets.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_prof.sh r4q2 c4 c5
