#!/bin/bash
# Round-4 session M: stacked shared-layer weight gradients -- linear / step / parity tests, C2 bench.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_step.py tests/test_gpu_mlp.py \
  tests/test_gpu_model_parity.py tests/test_gpu_dist_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 200 $O/bench.json
exit $rc
