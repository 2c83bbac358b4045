#!/bin/bash
# rocprofv3 kernel trace of a short graphed bench with the deferred expert wgrads
set -u
TAG=${1:-r2i}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-e2e-roofline --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err; rc=$?
echo "ROCPROF $rc"; head -c 200 $O/bench.json
exit $rc
