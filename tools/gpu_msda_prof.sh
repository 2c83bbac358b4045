TAG=${1:-msda}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/msda_probe.py > $O/probe.jsonl 2> $O/probe.err; rc=$?
echo "rc $rc"; cat $O/probe.jsonl
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'msda' in r['Name']: print(f"{float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>5}  {r['Name'][:90]}")
PY
