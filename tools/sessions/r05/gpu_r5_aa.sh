#!/bin/bash
# Round-5 session AA: bias-gradient column sum with 8 rows in flight and up to
# 512 blocks: linear tests, bench, kernel trace.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5aa; mkdir -p $O/prof; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_linear.py tests/test_gpu_step.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0 > $O/bench.json 2>> $O/bench.err; rc=$?
echo "BENCH $rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
