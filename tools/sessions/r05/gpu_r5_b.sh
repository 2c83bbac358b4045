#!/bin/bash
# Round-5 session B: drop-in test; conv forward ring-depth variants (conv_big
# 0..5) on the C2 shapes with a correctness check; C4 A/B of the per-layer
# lossless budget (default) vs every layer at 2x the mean (-epmb0) vs lossless (-epcf0).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5b; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dropin.py \
  > $O/pytest_dropin.log 2>&1; rc=$?
echo "PYTEST_DROPIN $rc"; tail -3 $O/pytest_dropin.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SH="8,256,256,46,80,3 8,256,256,92,160,3 8,128,128,92,160,3 8,512,512,23,40,3 8,1024,256,46,80,1 8,512,256,92,160,1 8,256,1024,46,80,1 8,256,256,92,160,3,2"
for m in 0 1 2 3 4 5; do
  timeout -k 10 240 python tools/conv_bench.py conv_big=$m $SH > $O/conv_big$m.jsonl 2> $O/conv_big$m.err; rc=$?
  echo "CONV_BIG $m $rc"
  [ $rc -eq 0 ] || exit $rc
done
for x in "" -epmb0 -epcf0; do
  timeout -k 10 420 python bench.py --workload c4 --spec-extra "$x" --no-cpu-baseline --no-e2e-roofline --steps 20 \
    --eval-steps 0 > $O/bench_c4$x.json 2> $O/bench_c4$x.err; rc=$?
  echo "BENCH_C4 $x $rc"; tail -c 300 $O/bench_c4$x.json
  [ $rc -eq 0 ] || exit $rc
done
