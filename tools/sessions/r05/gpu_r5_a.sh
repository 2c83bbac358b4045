#!/bin/bash
# Round-5 session A: the new / changed GPU tests (drop-in scripts on device 0,
# EP default slots + aux-path gradients, 2-rank lossy EP, router wgrad, MSDA),
# then C2 and C4 bench lines with the eval leg.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5a; mkdir -p $O; cd $R
MOE_PARITY_REPORT=$O/parity.json timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dropin.py tests/test_gpu_fullsize.py -k "dropin or ep_" tests/test_gpu_dist_graphs.py \
  > $O/pytest_new.log 2>&1; rc=$?
echo "PYTEST_NEW $rc"; tail -5 $O/pytest_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  -k "router_wgrad" tests/test_gpu_msda.py tests/test_gpu_step.py > $O/pytest_k.log 2>&1; rc=$?
echo "PYTEST_K $rc"; tail -3 $O/pytest_k.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 > $O/bench_c2.json 2> $O/bench_c2.err; rc=$?
echo "BENCH_C2 $rc"; tail -c 1500 $O/bench_c2.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --workload c4 --no-cpu-baseline --no-e2e-roofline --steps 20 > $O/bench_c4.json 2> $O/bench_c4.err; rc=$?
echo "BENCH_C4 $rc"; tail -c 800 $O/bench_c4.json
exit $rc
