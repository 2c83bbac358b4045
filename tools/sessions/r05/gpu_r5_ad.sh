#!/bin/bash
# Round-5 session AD: whole-detector parity at C2's batch 8 (bf16).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ad; mkdir -p $O; cd $R
MOE_PARITY_REPORT=$O/parity_b8.json timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_model_parity.py -k "8-720" > $O/tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 $O/tests.log
