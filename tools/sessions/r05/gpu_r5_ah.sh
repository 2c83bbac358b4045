#!/bin/bash
# Round-5 session AH: the HIP stem under bf16 autocast (evaluation forward):
# tests, eval A/B (MOE_STEM_HIP 2 / 0).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ah; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_conv.py -k stem tests/test_gpu_dropin.py tests/test_gpu_backbone.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 5 --warmup 2 --eval-steps 20"
for t in 2 0 2 0; do
  MOE_STEM_HIP=$t timeout -k 10 420 $B > $O/bench_s$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH stem=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
