#!/bin/bash
# Round-5 session E: C2 A/B of grouped-GEMM knobs on the new two-launch
# backward (heavy-group split-K, ring depths), and the PMC counter list.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5e; mkdir -p $O; cd $R
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "LIST $?"
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in "" "--tune wgrad_split_hot=12" "--tune wgrad_stages=3" "--tune gemm_stages=3" "" "--tune wgrad_split_hot=12" "--tune wgrad_stages=3" "--tune gemm_stages=3"; do
  timeout -k 10 420 $B $t > $O/bench_$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH [$t] $rc"
  [ $rc -eq 0 ] || exit $rc
done
