#!/bin/bash
# Round-5 session Z2: stem tests + kernel trace of the HIP stem (per-kernel durations).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5z2; mkdir -p $O/prof; cd $R
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_conv.py -k "stem or 32_channel" > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
MOE_STEM_HIP=2 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline --eval-steps 0 --steps 10 > $O/prof/bench.json 2> $O/prof/bench.err; rc=$?
echo "ROCPROF $rc"
