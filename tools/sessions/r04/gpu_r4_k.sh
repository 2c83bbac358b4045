#!/bin/bash
# Round-4 session K: BatchNorm statistics in the convolution epilogue -- tests, A/B (MOE_CONV_BN_STATS=0 as B).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bnact.py tests/test_gpu_step.py \
  tests/test_gpu_model_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh r4k_ab "MOE_CONV_BN_STATS=0"
