#!/bin/bash
# GPU call: LN / step / model-parity tests, then the C2 (default) and C4 bench lines.
set -u
TAG=${1:-r2f}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_kernels.py tests/test_gpu_step.py \
  tests/test_gpu_model_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err; rc=$?
echo "BENCH c2 $rc"; head -c 300 $O/bench_c2.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err; rc=$?
echo "BENCH c4 $rc"; head -c 300 $O/bench_c4.json; echo
exit $rc
