#!/bin/bash
# Round-4 session H: chunked router weight gradient -- tests, cold kbench, C2 bench line.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_r4.sh r4h "tests/test_gpu_kernels.py::test_router_wgrad_vs_fp64 tests/test_gpu_expert_ffn.py tests/test_gpu_fullsize.py tests/test_gpu_dist_graphs.py tests/test_gpu_step.py" router fkb
