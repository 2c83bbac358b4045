#!/bin/bash
# Round-5 session T: fold backward batched, value-projection casts, no token
# gradient fills; tests + bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5t; mkdir -p $O; cd $R
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 800 $T tests/test_gpu_fusions.py tests/test_gpu_backbone.py tests/test_gpu_model_parity.py tests/test_gpu_step.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 0 1 0; do
  MOE_FOLD_BWD_BATCH=$t timeout -k 10 420 $B > $O/bench_f$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH fold_batch=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
