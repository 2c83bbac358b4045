#!/bin/bash
# Round-4 bundle: torch profiler with source stacks (glue attribution), C4 + C5 bench lines, MSDA probe.
set -u
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r4n
timeout -k 10 400 python tools/torch_prof.py --stacks --steps 2 --out gpurun_out/r4n/tprof_stacks.txt > gpurun_out/r4n/tprof.log 2>&1; rc=$?
echo "TPROF $rc"
[ $rc -eq 0 ] || exit $rc
for WL in c4 c5; do
  timeout -k 10 420 python bench.py --workload $WL > gpurun_out/r4n/bench_$WL.json 2> gpurun_out/r4n/bench_$WL.err; rc=$?
  echo "BENCH $WL $rc"; tail -c 300 gpurun_out/r4n/bench_$WL.json
  [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_msda_prof.sh r4n_msda
