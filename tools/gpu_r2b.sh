#!/bin/bash
# Round-2 parity session: full-size layer + whole-detector parity (reports to
# gpurun_out/r2b/parity.json), then the whole GPU suite, then the bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r2b}; mkdir -p $O; cd $R
MOE_PARITY_REPORT=$O/parity.json timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_model_parity.py \
  -v --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
echo "PARITY $rc"; tail -25 $O/pytest_parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_model_parity.py > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; cat $O/bench.json
exit $rc
