#!/bin/bash
# Round-5 session N: 6-deep LDS-DMA ring for the long-K sub-chip row GEMMs
# (decoder GEMM2): exactness tests, kbench sweep, bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5n; mkdir -p $O; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
rc=0
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only gemm2_fwd --sweep deep_stages=3,4,6 \
  > $O/kbench_deep.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 3 6 4 3 6 4; do
  timeout -k 10 420 $B --tune deep_stages=$t > $O/bench_d$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH deep=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
