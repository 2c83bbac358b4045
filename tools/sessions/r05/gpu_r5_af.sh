#!/bin/bash
# Round-5 session AF: split BatchNorm finalizes (last-arriver merge): tests,
# bench A/B (bn_fin_split), kernel trace.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5af; mkdir -p $O/prof; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bnact.py tests/test_gpu_conv.py tests/test_gpu_fusions.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $T tests/test_gpu_model_parity.py tests/test_gpu_step.py tests/test_gpu_backbone.py > $O/tests2.log 2>&1; rc=$?
echo "TESTS2 $rc"; tail -2 $O/tests2.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 0 1 0; do
  timeout -k 10 420 $B --tune bn_fin_split=$t > $O/bench_f$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH split=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
