#!/bin/bash
# Per-launch expert-GEMM traffic (tools/gemm_traffic.py): one eager C2 bench
# step with the library's per-launch records dumped, and the same command
# under two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, no trace domains).
#   bash tools/gpu_gemm_traffic.sh <tag> [workload]
set -u
TAG=${1:-gt}; WL=${2:-c2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O/fetch $O/write
KRE="gemm_v|gemm_pair|gemm_triple|expert_ffn"
ARGS="--workload $WL --no-cpu-baseline --no-graphs --steps 1 --warmup 1 --eval-steps 0 --no-e2e-roofline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/fetch -o p -- \
  python3 $R/bench.py $ARGS --dump-prof-records $O/records.json > $O/fetch/bench.json 2> $O/fetch/bench.err; rc=$?
echo "FETCH $rc"
[ $rc -eq 0 ] || exit $rc
cp $O/records.json $O/records_fetch.json
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/write -o p -- \
  python3 $R/bench.py $ARGS --dump-prof-records $O/records.json > $O/write/bench.json 2> $O/write/bench.err; rc=$?
echo "WRITE $rc"
exit $rc
