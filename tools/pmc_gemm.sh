R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc1; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
K="python $R/multimodal-moe_amd/kbench.py --only gemm --variants 1,2 --stages 3 --rounds 1 --reps 3"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "gemm_v" --output-format csv -d $O/p1 -o p -- $K > $O/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "gemm_v" --output-format csv -d $O/p2 -o p -- $K > $O/p2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex "gemm_v" --output-format csv -d $O/p3 -o p -- $K > $O/p3.log 2>&1
echo DONE $?
