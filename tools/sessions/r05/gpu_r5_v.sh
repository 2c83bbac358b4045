#!/bin/bash
# Round-5 session V: 32-deep conv K-tiles (conv_k32 1-3: ring depth 2-4, up to
# 4 workgroups per CU): exactness tests, conv_bench per depth, bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5v; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_conv.py -k "k32 or bit_exact" > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py > $O/conv_k0.jsonl 2> $O/conv.err; rc=$?
echo "CONV k0 $rc"; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python tools/conv_bench.py conv_k32=$k > $O/conv_k$k.jsonl 2>> $O/conv.err; rc=$?
  echo "CONV k$k $rc"; [ $rc -eq 0 ] || exit $rc
done
