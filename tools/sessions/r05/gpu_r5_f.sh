#!/bin/bash
# Round-5 session F: PMC diagnosis of the conv forward body (3x3 256->256 at
# 92x160) and of the decoder grouped GEMMs; forward split-K A/B (kbench + bench).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5f; mkdir -p $O; cd $R
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only gemm2_fwd --sweep fwd_ksplit=0,2,4 \
  > $O/kbench_fwdsplit.jsonl 2> $O/kbench.err; rc=$?
echo "KBENCH_FWDSPLIT $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only ffn_bwd2 --skew 2.0 \
  > $O/kbench_bwd2_skew.jsonl 2>> $O/kbench.err; rc=$?
echo "KBENCH_BWD2 $rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VMEM TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
P3="TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "conv_fwd_kernel" --output-format csv -d $O/conv_p$i -o p -- \
    python3 $R/tools/conv_bench.py 8,256,256,92,160,3 > $O/conv_p$i.log 2>&1; rc=$?
  echo "PMC_CONV $i $rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "gemm_v2|gemm_triple" --output-format csv -d $O/gemm_p$i -o p -- \
    python3 $R/multimodal-moe_amd/kbench.py --rounds 1 --reps 5 --only gemm > $O/gemm_p$i.log 2>&1; rc=$?
  echo "PMC_GEMM $i $rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in "" "--tune fwd_ksplit=2" "" "--tune fwd_ksplit=2"; do
  timeout -k 10 420 $B $t > $O/bench_$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH [$t] $rc"; [ $rc -eq 0 ] || exit $rc
done
