#!/bin/bash
# Round-5 session O: time attribution of the decoder grouped GEMMs
# (gemm_debug 1: no C stores, 2: no main loop).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5o; mkdir -p $O; cd $R
for k in gemm1_fwd gemm2_fwd gemm_dgrad1 gemm_wgrad1; do
  timeout -k 10 300 python multimodal-moe_amd/kbench.py --rounds 3 --reps 30 --only $k --debug 0,1,2 \
    > $O/kbench_$k.jsonl 2>> $O/kbench.err; rc=$?
  echo "KBENCH $k $rc"; [ $rc -eq 0 ] || exit $rc
done
