#!/bin/bash
# rocprofv3 kernel-trace of kbench entries (true per-kernel durations, no event stamps):
#   bash tools/gpu_kprof.sh <tag> <kbench --only filter> [extra kbench args]
set -u
TAG=$1; ONLY=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/multimodal-moe_amd/kbench.py --rounds 1 --reps 20 --only $ONLY "$@" > $O/kbench.jsonl 2> $O/kbench.err; rc=$?
echo "KPROF $rc"
[ $rc -eq 0 ] || exit $rc
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>5}  {r['Name'][:100]}")
PY
