#!/bin/bash
# Round-end style check: the GPU test suite, smoke(), the default bench line,
# then (optional, extra args) a kernel microbenchmark run.
#   bash tools/gpu_check.sh <tag> [kbench args...]
set -u
TAG=${1:-chk}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
MOE_TEST_MEMLOG=$O/memlog.txt MOE_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v \
  --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "SMOKE $rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 300 $O/bench.json
[ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 400 python multimodal-moe_amd/kbench.py "$@" > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
  echo "KBENCH $rc"
fi
exit $rc
