#!/bin/bash
# Round-4 session I: router wgrad merge batching, conv pair, compaction tail, aux views -- tests, kprof A/B, C2 bench.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_kernels.py::test_router_wgrad_vs_fp64 tests/test_gpu_conv.py \
  tests/test_gpu_expert_ffn.py tests/test_gpu_step.py tests/test_gpu_dist_graphs.py tests/test_gpu_model_parity.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -3 $O/first.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_kprof.sh r4i/kp1 router_wgrad && bash tools/gpu_kprof.sh r4i/kp0 router_wgrad --tune router_wgrad_chunked=0 || exit 1
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 300 $O/bench.json
exit $rc
