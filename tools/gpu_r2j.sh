#!/bin/bash
# GPU call: side-stream expert weight gradients (MOE_DEFER_MOE_WGRAD=2) -- tests, then an interleaved A/B
set -u
TAG=${1:-r2j}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "deferred" -m gpu -q -x --timeout 200 \
  --timeout-method thread > $O/pytest_k.log 2>&1; rc=$?
echo "PYTEST_K $rc"; tail -2 $O/pytest_k.log
[ $rc -eq 0 ] || exit $rc
MOE_DEFER_MOE_WGRAD=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -q -x --timeout 200 \
  --timeout-method thread > $O/pytest_s.log 2>&1; rc=$?
echo "PYTEST_S $rc"; tail -2 $O/pytest_s.log
[ $rc -eq 0 ] || exit $rc
for f in 0 2 0 2; do
  MOE_DEFER_MOE_WGRAD=$f timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline > $O/bench_d$f.json 2> $O/bench_d$f.err; rc=$?
  echo "BENCH defer=$f $rc"; head -c 160 $O/bench_d$f.json; echo
  [ $rc -eq 0 ] || exit $rc
  cat $O/bench_d$f.json >> $O/bench_all.jsonl
done
exit 0
