#!/bin/bash
# Round-5 session D: moe_expert_ffn_bwd equality tests, graphed eval forward
# test, the MoE layer tests; C2 A/B of the two-launch expert FFN backward
# (MOE_FFN_BWD2=1 default vs 0 = paired launches), eval leg.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5d; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_expert_ffn.py \
  tests/test_gpu_dropin.py tests/test_gpu_kernels.py -k "ffn or dropin or eval_forward or moe_layer" \
  > $O/pytest.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20"
for v in 1 0 1 0; do
  MOE_FFN_BWD2=$v timeout -k 10 420 $B --eval-steps 10 > $O/bench_c2_bwd2_$v.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH_C2 bwd2=$v $rc"
  [ $rc -eq 0 ] || exit $rc
done
