#!/bin/bash
# Round-5 session AG: kernel trace of the graphed eval forward (bench eval leg).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ag2; mkdir -p $O/prof; cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-kernel-timing --steps 2 --warmup 1 --eval-steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
