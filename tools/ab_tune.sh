#!/bin/bash
# Interleaved A/B of one libmoe_hip tuning knob on the default bench:
#   bash tools/ab_tune.sh <tag> <key> <valueB> [bench args...]
# runs A (default), B (--tune key=valueB), A, B; prints images/s.
set -u
TAG=$1; KEY=$2; VB=$3; shift 3
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O/db
cp $GRAFT_REPO_ROOT/multimodal-moe_amd/miopen_db/*.txt $O/db/
export MIOPEN_USER_DB_PATH=$O/db
cd $GRAFT_REPO_ROOT
for r in a1 b1 a2 b2; do
  T=""; [ "${r:0:1}" = "b" ] && T="--tune $KEY=$VB"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --eval-steps 0 $T "$@" > $O/$r.json 2> $O/$r.err || exit $?
  python3 -c "import json;b=json.load(open('$O/$r.json'));print('$r $KEY', b['value'], b['ms_per_step'], b['roofline'].get('avg_us'))"
done
