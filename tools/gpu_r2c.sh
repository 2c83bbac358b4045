#!/bin/bash
# Round-2 (session 3) GPU call: round-end style check on the current library,
# a kernel A/B of the backward GEMM pairs against lib/libmoe_hip_base.so
# (the previous commit's kernels), an end-to-end A/B bench, then glue-op attribution.
#   bash tools/gpu_r2c.sh <tag>
set -u
TAG=${1:-r2c}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
BASE=$R/multimodal-moe_amd/lib/libmoe_hip_base.so
bash tools/gpu_check.sh $TAG/chk || exit $?
for v in base new; do
  if [ $v = base ]; then export MOE_HIP_LIB=$BASE; else unset MOE_HIP_LIB; fi
  timeout -k 10 300 python multimodal-moe_amd/kbench.py --only gemm > $O/kbench_$v.jsonl 2> $O/kbench_$v.err; rc=$?
  echo "KBENCH $v $rc"; cat $O/kbench_$v.jsonl
  [ $rc -eq 0 ] || exit $rc
done
for v in base new; do
  if [ $v = base ]; then export MOE_HIP_LIB=$BASE; else unset MOE_HIP_LIB; fi
  timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  echo "BENCH $v $rc"; head -c 400 $O/bench_$v.json; echo
  [ $rc -eq 0 ] || exit $rc
done
unset MOE_HIP_LIB
timeout -k 10 300 python -u tools/torch_prof.py --stacks --steps 2 --warmup 3 --out $O/tprof_stacks.txt \
  > $O/tprof.log 2>&1; rc=$?
echo "TPROF $rc"; tail -3 $O/tprof.log
exit $rc
