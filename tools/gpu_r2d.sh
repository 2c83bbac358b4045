#!/bin/bash
# GPU call: GPU suite, kernel A/B of the grouped GEMMs against
# lib/libmoe_hip_base.so (previous grouped_gemm.o), e2e A/B of the fused
# residual + fused LayerNorm (MOE_FUSE_RESIDUAL / MOE_FUSED_LN = 0/1).   bash tools/gpu_r2d.sh <tag>
set -u
TAG=${1:-r2d}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
BASE=$R/multimodal-moe_amd/lib/libmoe_hip_base.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in base new; do
  if [ $v = base ]; then export MOE_HIP_LIB=$BASE; else unset MOE_HIP_LIB; fi
  timeout -k 10 300 python multimodal-moe_amd/kbench.py --only gemm > $O/kbench_$v.jsonl 2> $O/kbench_$v.err; rc=$?
  echo "KBENCH $v $rc"
  [ $rc -eq 0 ] || exit $rc
done
unset MOE_HIP_LIB
for f in 0 1 0 1; do
  MOE_FUSE_RESIDUAL=$f MOE_FUSED_LN=$f timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline > $O/bench_f$f.json 2> $O/bench_f$f.err; rc=$?
  echo "BENCH fuse=$f $rc"; head -c 200 $O/bench_f$f.json; echo
  [ $rc -eq 0 ] || exit $rc
  cat $O/bench_f$f.json >> $O/bench_all.jsonl
done
exit 0
