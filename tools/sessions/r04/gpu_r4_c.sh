#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_r4.sh r4q "tests/test_gpu_fullsize.py tests/test_gpu_mlp.py tests/test_gpu_step.py tests/test_gpu_dist_graphs.py tests/test_gpu_expert_ffn.py" "" f; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4q c2
