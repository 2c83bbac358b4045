#!/bin/bash
# Round-5 session Z: the frozen stem on libmoe_hip (direct 3 -> 32 kernel;
# mode 2 also the 32-channel implicit GEMMs): tests, bench A/B (MOE_STEM_HIP
# 1 / 2 / 0), kernel trace of mode 1.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5z; mkdir -p $O/prof; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_conv.py tests/test_gpu_backbone.py tests/test_gpu_model_parity.py tests/test_gpu_dropin.py tests/test_gpu_step.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 10"
for t in 2 0 2 0; do
  MOE_STEM_HIP=$t timeout -k 10 420 $B > $O/bench_s$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH stem=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
MOE_STEM_HIP=2 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
