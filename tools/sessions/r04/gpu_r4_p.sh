#!/bin/bash
# Round-4 session P: C2 A/B of the fused expert FFN (B = never fused).
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/ab_env.sh r4p_ab "MOE_FUSED_FFN_MIN_ROWS=1000000"
