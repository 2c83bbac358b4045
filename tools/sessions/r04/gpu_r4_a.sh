#!/bin/bash
# Round-4 session A: full GPU suite (parity report), C2 bench line, conv A/B of the 256 x 256 tile.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_r4.sh r4p "" "" pb; rc=$?
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_conv_ab.sh r4p_conv conv_big=2
