#!/bin/bash
# One rocprofv3 kernel-trace run of the default bench (graph replay) for a
# per-kernel step breakdown (tools/step_breakdown.py):  bash tools/gpu_trace_c2.sh <tag> [bench args]
set -u
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 "$@" > $O/bench.json 2> $O/bench.err; rc=$?
echo "TRACE $rc"
exit $rc
