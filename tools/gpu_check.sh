#!/bin/bash
# Round-end style check: the GPU test suite, smoke(), the default bench line.
#   bash tools/gpu_check.sh <tag>
set -u
TAG=${1:-chk}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
MOE_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 300 $O/bench.json
exit $rc
