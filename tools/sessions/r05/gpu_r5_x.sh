#!/bin/bash
# Round-5 session X: PyTorch TunableOp over the step's hipBLASLt / rocBLAS
# GEMMs (value projection, decoder linears): tune once in the eager warm-up,
# then A/B the graphed step with the tuned table against the library default.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5x; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e-roofline --eval-steps 0"
export PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
  timeout -k 10 700 $B --steps 5 --warmup 2 > $O/tune.json 2> $O/tune.err; rc=$?
echo "TUNE $rc"; ls -la $O; [ $rc -eq 0 ] || exit $rc
for t in 1 0 1 0; do
  PYTORCH_TUNABLEOP_ENABLED=$t PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 420 $B --steps 20 > $O/bench_t$t.$RANDOM.json 2>> $O/bench.err; rc=$?
  echo "BENCH tunableop=$t $rc"; [ $rc -eq 0 ] || exit $rc
done
