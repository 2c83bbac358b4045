#!/bin/bash
# PMC passes over the HIP convolution kernels of one conv_bench shape (separate runs, no trace domains):
#   bash tools/pmc_conv.sh <tag> <shape e.g. 8,256,256,92,160,3> [tuning k=v ...]
set -u
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
K="python3 $R/tools/conv_bench.py $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "conv_fwd_kernel|conv_wgrad_kernel" --output-format csv \
    -d $O/p$i -o p -- $K > $O/p$i.log 2>&1; rc=$?
  echo "PASS $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - $O <<'PY'
import csv, sys, glob
from collections import defaultdict
O = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
for f in glob.glob(O + "/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void moe::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add(r.get("Dispatch_Id"))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        n = max(1, len(cnt[(k, c)]))
        print(f"   {c:28s} {v / n:16.1f} per dispatch")
PY
