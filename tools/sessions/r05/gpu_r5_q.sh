#!/bin/bash
# Round-5 session Q: glue census (all sizes) + clean kernel trace after the fusions.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5q; mkdir -p $O/prof; cd $R
CENSUS_MIN_NUMEL=1000 timeout -k 10 400 python tools/glue_census.py > $O/census.txt 2> $O/census.err; rc=$?
echo "CENSUS $rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 --no-kernel-timing > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"; exit $rc
