#!/bin/bash
# GPU call: the deferred expert weight gradients -- parity tests, then an
# interleaved end-to-end A/B (MOE_DEFER_MOE_WGRAD = 0 / 1).
set -u
TAG=${1:-r2h}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "deferred or residual or layer_fwd_bwd or bwd_pair" \
  -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_k.log 2>&1; rc=$?
echo "PYTEST_K $rc"; tail -3 $O/pytest_k.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_model_parity.py tests/test_gpu_dist_graphs.py \
  -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_s.log 2>&1; rc=$?
echo "PYTEST_S $rc"; tail -3 $O/pytest_s.log
[ $rc -eq 0 ] || exit $rc
for f in 0 1 0 1; do
  MOE_DEFER_MOE_WGRAD=$f timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline > $O/bench_d$f.json 2> $O/bench_d$f.err; rc=$?
  echo "BENCH defer=$f $rc"; head -c 200 $O/bench_d$f.json; echo
  [ $rc -eq 0 ] || exit $rc
  cat $O/bench_d$f.json >> $O/bench_all.jsonl
done
exit 0
