#!/bin/bash
# Round-4 session V: GradLink through downsampling shortcuts -- tests, C2 A/B (B = relu_grad2).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_backbone.py tests/test_gpu_model_parity.py tests/test_gpu_step.py \
  tests/test_gpu_dist_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh r4v_ab "MOE_DOWN_LINK=0"
