#!/bin/bash
# L2 behaviour of the grouped-GEMM kernels on the kbench shapes (one PMC group per pass).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcw; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
K="python3 $R/multimodal-moe_amd/kbench.py --only gemm --variants 2 --stages 2 --rounds 1 --reps 5"
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex "gemm_v2" --output-format csv -d $O/p1 -o p -- $K > $O/p1.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_REQ_sum --kernel-include-regex "gemm_v2" --output-format csv -d $O/p2 -o p -- $K > $O/p2.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --kernel-include-regex "gemm_v2" --output-format csv -d $O/p3 -o p -- $K > $O/p3.log 2>&1
echo DONE $?
