#!/bin/bash
# Round-5 session C: hipBLASLt GEMM reference at the conv GEMM shapes; C4 A/B of
# the per-layer lossless budget; C2 A/B of heavy-group split-K for the decoder
# weight gradients (wgrad_split_hot).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5c; mkdir -p $O; cd $R
SH="8,256,256,46,80,3 8,256,256,92,160,3 8,128,128,92,160,3 8,512,512,23,40,3 8,1024,256,46,80,1 8,512,256,92,160,1 8,256,1024,46,80,1 8,64,256,184,320,1 8,64,64,184,320,3"
timeout -k 10 240 python tools/conv_bench.py $SH > $O/conv_ref.jsonl 2> $O/conv_ref.err; rc=$?
echo "CONV_REF $rc"
[ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for x in "" "--spec-extra=-epmb0" "--spec-extra=-epcf0" ""; do
  timeout -k 10 420 $B --workload c4 $x > $O/bench_c4_$RANDOM.json 2>> $O/bench_c4.err; rc=$?
  echo "BENCH_C4 [$x] $rc"
  [ $rc -eq 0 ] || exit $rc
done
for t in 0 12 10 0 12 10; do
  timeout -k 10 420 $B --tune wgrad_split_hot=$t > $O/bench_c2_hot$t.$RANDOM.json 2>> $O/bench_c2.err; rc=$?
  echo "BENCH_C2 hot=$t $rc"
  [ $rc -eq 0 ] || exit $rc
done
