#!/bin/bash
# GPU call: kernel parity tests, router A/B (kbench, base = previous router),
# then the C5 profile (bench + rocprof + PMC passes via gpu_prof.sh).
set -u
TAG=${1:-r2g}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
BASE=$R/multimodal-moe_amd/lib/libmoe_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_mx.py \
  -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in c2 c5; do
for v in base new; do
  if [ $v = base ]; then export MOE_HIP_LIB=$BASE; else unset MOE_HIP_LIB; fi
  timeout -k 10 200 python multimodal-moe_amd/kbench.py --only router --config $cfg > $O/kbench_router_${cfg}_$v.jsonl 2> $O/kbench_$v.err; rc=$?
  echo "KBENCH $cfg $v $rc"; cat $O/kbench_router_${cfg}_$v.jsonl
  [ $rc -eq 0 ] || exit $rc
done
done
unset MOE_HIP_LIB
bash tools/gpu_prof.sh $TAG c5
