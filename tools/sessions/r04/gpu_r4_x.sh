#!/bin/bash
# Round-4 session X: combined A/B of this round's late glue work (B = all of it off).
set -u
R=$GRAFT_REPO_ROOT; cd $R
bash tools/ab_env.sh r4x_ab "MOE_CONV_PAIR=0 MOE_CONV_BN_STATS=0 MOE_LN_POS=0 MOE_DOWN_LINK=0 MOE_BATCHED_FLIPS=0"
