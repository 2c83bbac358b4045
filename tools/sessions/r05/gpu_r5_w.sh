#!/bin/bash
# Round-5 session W: automatic 32-deep K-tiles for wide 1x1 convolutions
# (conv_k32 = -1): conv tests, conv_bench, bench A/B against conv_k32=0.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5w; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_conv.py tests/test_gpu_backbone.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py > $O/conv_auto.jsonl 2> $O/conv.err; rc=$?
echo "CONV auto $rc"; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in -1 0 -1 0; do
  timeout -k 10 420 $B --tune conv_k32=$t > $O/bench_k$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH k32=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
