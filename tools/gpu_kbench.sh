#!/bin/bash
# GPU session for kernel work: GPU parity tests, then the kernel microbenchmark,
# then the default bench line.  bash tools/gpu_kbench.sh <tag> [kbench args...]
set -u
TAG=${1:-kb}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 420 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python multimodal-moe_amd/kbench.py "$@" > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"; cat $O/kbench.jsonl; tail -3 $O/kbench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; cat $O/bench.json; tail -3 $O/bench.err
exit $rc
