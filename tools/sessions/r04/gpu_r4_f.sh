#!/bin/bash
# Round-4 session F: batched-flip tests + graph tests, C2 bench line, the C5 profile set.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_r4.sh r4f2 "tests/test_gpu_conv.py tests/test_gpu_step.py tests/test_gpu_dist_graphs.py tests/test_gpu_graph_topology.py tests/test_gpu_mlp.py" "" fb; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4f2 c5
