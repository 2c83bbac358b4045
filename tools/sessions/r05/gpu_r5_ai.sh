#!/bin/bash
# Round-5 session AI: inference-mode BatchNorm in one HIP pass
# (rtdetr_bn_act_eval): tests, eval A/B (MOE_BN_EVAL).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ai; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 800 $T tests/test_gpu_bnact.py tests/test_gpu_dropin.py tests/test_gpu_model_parity.py tests/test_gpu_backbone.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 10 --warmup 2 --eval-steps 20"
for t in 1 0 1 0; do
  MOE_BN_EVAL=$t timeout -k 10 420 $B > $O/bench_e$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH bn_eval=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
