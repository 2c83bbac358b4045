#!/bin/bash
# Round-5 session S: convolution A operand in registers (conv_areg): exactness
# tests, conv_bench A/B at the C2 shapes, bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5s; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_conv.py -k "areg" > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py > $O/conv_off.jsonl 2> $O/conv.err; rc=$?
echo "CONV off $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py conv_areg=1 conv_bm=128 > $O/conv_on.jsonl 2>> $O/conv.err; rc=$?
echo "CONV on $rc"; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 0 1 0; do
  timeout -k 10 420 $B --tune conv_areg=$t > $O/bench_a$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH areg=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
