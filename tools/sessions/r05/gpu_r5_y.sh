#!/bin/bash
# Round-5 session Y: slot-major BatchNorm partials with one-wave-per-channel
# finalize kernels; narrow head linears (rtdetr_linear_narrow_*): tests,
# bench A/B (MOE_NARROW_LINEAR), kernel trace.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5y; mkdir -p $O/prof; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_bnact.py tests/test_gpu_conv.py tests/test_gpu_fusions.py tests/test_gpu_backbone.py \
  tests/test_gpu_model_parity.py tests/test_gpu_step.py tests/test_gpu_mlp.py tests/test_gpu_linear.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 0 1 0; do
  MOE_NARROW_LINEAR=$t timeout -k 10 420 $B > $O/bench_n$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH narrow=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
