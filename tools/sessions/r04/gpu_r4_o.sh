#!/bin/bash
# Round-4 session O: EP two-launch forward -- tests, C4 A/B (B = fused FFN everywhere).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_expert_ffn.py tests/test_gpu_dist_graphs.py tests/test_gpu_step.py \
  tests/test_gpu_fullsize.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh r4o_ab "MOE_FUSED_FFN_MIN_ROWS=0" --workload c4
