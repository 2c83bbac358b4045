#!/bin/bash
# Round-4 session T: LayerNorm + pos -- tests, C2 A/B (B = separate add).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_model_parity.py tests/test_gpu_step.py \
  tests/test_gpu_dist_graphs.py tests/test_gpu_graph_topology.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh r4t_ab "MOE_LN_POS=0"
