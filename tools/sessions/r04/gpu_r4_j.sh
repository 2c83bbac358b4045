#!/bin/bash
# Round-4 session J: conv pair A/B (MOE_CONV_PAIR=0 as B), then the whole GPU suite.
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/ab_env.sh r4j_ab "MOE_CONV_PAIR=0" || exit $?
bash tools/gpu_r4.sh r4j "" "" p
