#!/bin/bash
# Round-4 development session: new-kernel tests first (stop on a fault), then
# kernel microbenchmarks (MoE GEMMs cold; convolutions A/B of the 8-wave tile),
# the whole GPU suite and the default bench line.
#   bash tools/gpu_r4.sh <tag> [pytest targets] [kbench --only filter] [stages: any of f k c p b]
set -u
TAG=${1:-r4}; FIRST=${2:-tests/test_gpu_expert_ffn.py}; ONLY=${3:-}; ST=${4:-fkcpb}
on() { [[ $ST == *$1* ]]; }
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
fatal() { [ $1 -ge 2 ] && [ $1 -ne 5 ]; }   # pytest: 0 ok, 1 failures, 5 none collected
on f && { timeout -k 10 420 python -u -m pytest $FIRST -m gpu -x -v --timeout 120 --timeout-method thread > $O/first.log 2>&1; rc=$?
echo "FIRST $rc"; tail -5 $O/first.log
[ $rc -eq 0 ] || exit $rc; }
on k && { timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 20 --cold ${ONLY:+--only $ONLY} > $O/kbench_cold.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"
[ $rc -eq 0 ] || exit $rc; }
on c && { CS="8,256,256,46,80,3 8,256,256,92,160,3 8,256,256,23,40,3 8,128,128,92,160,3 8,512,512,23,40,3 8,1024,256,46,80,1 8,512,256,92,160,1 8,256,256,92,160,3,2"
timeout -k 10 300 python tools/conv_bench.py $CS > $O/conv_default.jsonl 2> $O/conv.err && \
timeout -k 10 300 python tools/conv_bench.py conv_big=1 $CS > $O/conv_big.jsonl 2>> $O/conv.err; rc=$?
echo "CONV $rc"
[ $rc -eq 0 ] || exit $rc; }
on p && { MOE_TEST_MEMLOG=$O/memlog.txt MOE_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -4 $O/pytest_gpu.log
fatal $rc && exit $rc; }
on b || exit 0
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; tail -c 600 $O/bench.json
exit $rc
