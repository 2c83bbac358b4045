#!/bin/bash
# Round-5 session AC: query-selection top-k on libmoe_hip (rtdetr_topk_rows):
# tests, bench A/B (MOE_HIP_TOPK), eval leg.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ac; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_fusions.py tests/test_gpu_model_parity.py tests/test_gpu_msda.py tests/test_gpu_dropin.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 10"
for t in 1 0 1 0; do
  MOE_HIP_TOPK=$t timeout -k 10 420 $B > $O/bench_t$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH topk=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
