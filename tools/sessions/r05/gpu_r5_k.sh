#!/bin/bash
# Round-5 session K: dense-linear probe (hipBLASLt vs libmoe_hip dense GEMM).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5k; mkdir -p $O; cd $R
timeout -k 10 300 python tools/linear_probe.py > $O/probe.jsonl 2> $O/probe.err; rc=$?
echo "PROBE $rc"; exit $rc
