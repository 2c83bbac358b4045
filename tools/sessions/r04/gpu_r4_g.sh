#!/bin/bash
# Round-4 session G: glue attribution (C2 by input shape, C4 by source line), then the C4 profile set.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4g2
timeout -k 10 400 python tools/torch_prof.py --glue-shapes --steps 2 --out gpurun_out/r4g2/tprof_c2_shapes.txt \
  > gpurun_out/r4g2/tprof_c2.log 2>&1; rc=$?
echo "TPROF C2 $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/torch_prof.py --stacks --spec rtdetr-r50-moe16-top2-ep1 --single-ctx --steps 2 \
  --out gpurun_out/r4g2/tprof_c4_stacks.txt > gpurun_out/r4g2/tprof_c4.log 2>&1; rc=$?
echo "TPROF C4 $rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r4g2 c4
