#!/bin/bash
# Round-5 session AB: small-K narrow forward (weights in registers, rows
# strided), tests, bench; glue census of the small torch ops.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ab; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_fusions.py tests/test_gpu_mlp.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0 > $O/bench.json 2>> $O/bench.err; rc=$?
echo "BENCH $rc"; [ $rc -eq 0 ] || exit $rc
CENSUS_MIN_NUMEL=1 timeout -k 10 300 python tools/glue_census.py > $O/census.txt 2> $O/census.err; rc=$?
echo "CENSUS $rc"
