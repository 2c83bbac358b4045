#!/bin/bash
# One GPU session (round 2): the GPU test suite (parity reports to
# gpurun_out/<tag>/parity*.json), the default bench line, the kernel
# microbenchmark.  bash tools/gpu_session.sh <tag> [kbench args...]
set -u
TAG=${1:-s}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
MOE_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 600 $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python multimodal-moe_amd/kbench.py "$@" > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"
exit $rc
