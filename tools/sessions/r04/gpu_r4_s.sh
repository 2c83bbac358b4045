#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4s
timeout -k 10 200 python tools/vproj_probe.py > gpurun_out/r4s/vproj.jsonl 2> gpurun_out/r4s/vproj.err; rc=$?
echo "PROBE $rc"; cat gpurun_out/r4s/vproj.jsonl; tail -3 gpurun_out/r4s/vproj.err
exit $rc
