#!/bin/bash
# Round-5 session L: stage-output gradients through the GradLink (stage taps),
# fork without materialised zero gradients, level memory, selection rows in
# the value projection; the round-4 path for the record; A/B bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5l; mkdir -p $O; cd $R
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
MOE_STAGE_TAP=0 timeout -k 10 300 $T tests/test_gpu_backbone.py -k external_consumer > $O/old_path.log 2>&1; echo "OLD_PATH $? (expected to fail: the round-4 gradient)"
timeout -k 10 700 $T tests/test_gpu_fusions.py tests/test_gpu_backbone.py tests/test_gpu_conv.py tests/test_gpu_model_parity.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 0 1 0; do
  MOE_STAGE_TAP=$t MOE_LEVEL_MEMORY=$t timeout -k 10 420 $B > $O/bench_new$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH new=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
