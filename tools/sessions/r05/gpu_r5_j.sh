#!/bin/bash
# Round-5 session J: torch-op census of one eager C2 step (launch floor).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5j; mkdir -p $O; cd $R
timeout -k 10 400 python tools/glue_census.py > $O/census.txt 2> $O/census.err; rc=$?
echo "CENSUS $rc"; exit $rc
