#!/bin/bash
# Round-5 session H: moe_expert_ffn_bwd shape rule (encoder back to the paired
# launches above bwd2_max_rows rows/expert) and the unsplit-dXp A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O; cd $R
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only ffn_bwd2 --sweep bwd2_max_rows=1024,1000000 \
  > $O/kbench_rows.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH_ROWS $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only ffn_bwd2 --sweep bwd2_dx_split=0,1 \
  > $O/kbench_dx.jsonl 2>> $O/kbench.err; rc=$?
echo "KBENCH_DX $rc"; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in "" "--tune bwd2_max_rows=1000000" "--tune bwd2_dx_split=1" "" "--tune bwd2_max_rows=1000000" "--tune bwd2_dx_split=1"; do
  timeout -k 10 420 $B $t > $O/bench_$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH [$t] $rc"; [ $rc -eq 0 ] || exit $rc
done
