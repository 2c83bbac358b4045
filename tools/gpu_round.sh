#!/bin/bash
# One GPU session: parity tests, the default bench line, a rocprofv3 kernel-trace
# summary of the same bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE)
# over the MoE kernels for the roofline `traffic` field.  Usage (on the box):
#   bash tools/gpu_round.sh <tag>
# Every GPU step has its own time limit; the script stops at the first step that
# faults, aborts or times out (exit status >= 2 other than a pytest failure).
set -u
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O/prof $O/pmc_fetch $O/pmc_write
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }

cd $R
timeout -k 10 420 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -3 $O/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 420 python bench.py --phase-timing > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"; cat $O/prof/bench.json
[ $rc -eq 0 ] || exit $rc
KRE="gemm_v|permute_fwd|combine_fwd|combine_bwd|router_topk|token_bwd|msda_"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_fetch -o p -- \
  python3 $R/bench.py --no-cpu-baseline --no-kernel-timing --no-graphs --steps 3 --warmup 1 > $O/pmc_fetch/bench.json 2> $O/pmc_fetch/bench.err; rc=$?
echo "PMC_FETCH $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_write -o p -- \
  python3 $R/bench.py --no-cpu-baseline --no-kernel-timing --no-graphs --steps 3 --warmup 1 > $O/pmc_write/bench.json 2> $O/pmc_write/bench.err; rc=$?
echo "PMC_WRITE $rc"
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 20 > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH $rc"
exit $rc
