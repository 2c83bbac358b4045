#!/bin/bash
# Profiling session (round 2+): per workload, the bench line, a rocprofv3
# kernel-trace summary of the same bench command, and two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs, no trace domains) over the MoE /
# MSDA kernels for the roofline `traffic` field.  Usage (on the box):
#   bash tools/gpu_prof.sh <tag> c2 c5 ...
# Summarise afterwards with: python tools/profile_summary.py gpurun_out/<tag>/<wl> profiles/<round>/<wl> <wl>
# Every GPU step has its own time limit; the script stops at the first failure.
# BENCH_EXTRA (env) is appended to every bench command (e.g. "--tune xcd_map=2").
set -u
X=${BENCH_EXTRA:-}
TAG=${1:-prof}; shift
R=$GRAFT_REPO_ROOT
KRE="conv_|attn_|gemm_v|gemm_pair|gemm_triple|expert_ffn|router_wgrad|ep_compaction|permute_fwd|combine_fwd|combine_bwd|router_topk|route_dispatch|route_index|route_scan|token_bwd|quantize_mx|msda_|linear_wgrad"
for WL in "$@"; do
  O=$R/gpurun_out/$TAG/$WL
  mkdir -p $O/prof $O/pmc_fetch $O/pmc_write
  cd $R
  timeout -k 10 420 python bench.py --workload $WL $X > $O/bench.json 2> $O/bench.err; rc=$?
  echo "BENCH $WL $rc"; tail -c 400 $O/bench.json
  [ $rc -eq 0 ] || exit $rc
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $R/bench.py --workload $WL --no-cpu-baseline --eval-steps 0 $X > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
  echo "ROCPROF $WL $rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_fetch -o p -- \
    python3 $R/bench.py --workload $WL --no-cpu-baseline --no-kernel-timing --no-graphs --steps 3 --warmup 1 --eval-steps 0 $X \
    > $O/pmc_fetch/bench.json 2> $O/pmc_fetch/bench.err; rc=$?
  echo "PMC_FETCH $WL $rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_write -o p -- \
    python3 $R/bench.py --workload $WL --no-cpu-baseline --no-kernel-timing --no-graphs --steps 3 --warmup 1 --eval-steps 0 $X \
    > $O/pmc_write/bench.json 2> $O/pmc_write/bench.err; rc=$?
  echo "PMC_WRITE $WL $rc"
  [ $rc -eq 0 ] || exit $rc
  # MFMA utilisation of the expert GEMMs from counters (one pass, no trace domains)
  mkdir -p $O/pmc_mfma
  timeout -k 10 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
    --kernel-include-regex "gemm_v|gemm_pair|gemm_triple|expert_ffn" --output-format csv -d $O/pmc_mfma -o p -- \
    python3 $R/bench.py --workload $WL --no-cpu-baseline --no-kernel-timing --no-graphs --steps 3 --warmup 1 --eval-steps 0 $X \
    > $O/pmc_mfma/bench.json 2> $O/pmc_mfma/bench.err; rc=$?
  echo "PMC_MFMA $WL $rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
