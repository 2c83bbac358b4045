#!/bin/bash
# Round-4 development session: new-kernel tests first (stop on a fault), then
# kernel microbenchmarks, the whole GPU suite and the default bench line.
#   bash tools/gpu_r4.sh <tag> [pytest target (default: tests/test_gpu_expert_ffn.py)] [kbench --only filter]
set -u
TAG=${1:-r4}; FIRST=${2:-tests/test_gpu_expert_ffn.py}; ONLY=${3:-}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
fatal() { [ $1 -ge 2 ] && [ $1 -ne 5 ]; }   # pytest: 0 ok, 1 failures, 5 none collected
timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -5 $O/first.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 20 --cold ${ONLY:+--only $ONLY} > $O/kbench_cold.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"
[ $rc -eq 0 ] || exit $rc
MOE_TEST_MEMLOG=$O/memlog.txt MOE_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest_gpu.log
fatal $rc && exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 600 $O/bench.json
exit $rc
