#!/bin/bash
# Round-5 session I: a clean training-only kernel trace of C2 (launch census).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5i; mkdir -p $O/prof; cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"; exit $rc
