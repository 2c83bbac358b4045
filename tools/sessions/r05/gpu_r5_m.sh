#!/bin/bash
# Round-5 session M: CSPRep shortcut add in the BatchNorm pass, dual linear
# for the deformable-attention heads, GradSlot between the encoder's
# downsampling convs and the decoder's input projections; tests + bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5m; mkdir -p $O; cd $R
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 800 $T tests/test_gpu_fusions.py tests/test_gpu_model_parity.py tests/test_gpu_step.py tests/test_gpu_dropin.py > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-e2e-roofline --steps 20 --eval-steps 0"
for t in 1 2 3; do
  timeout -k 10 420 $B > $O/bench_$t.json 2>> $O/bench.err; rc=$?
  echo "BENCH $t $rc"; [ $rc -eq 0 ] || exit $rc
done
