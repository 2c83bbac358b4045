#!/bin/bash
# A/B of an environment switch on one box with one shared MIOpen db copy:
#   bash tools/ab_env.sh <tag> "<env for B>" [bench args...]
# runs bench A (default env), B (with the env), A again.
set -u
TAG=$1; ENVB=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O/db
cp $GRAFT_REPO_ROOT/multimodal-moe_amd/miopen_db/*.txt $O/db/
export MIOPEN_USER_DB_PATH=$O/db
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > $O/a1.json 2> $O/a1.err || exit $?
timeout -k 10 300 env $ENVB python bench.py --no-cpu-baseline --steps 20 "$@" > $O/b.json 2> $O/b.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > $O/a2.json 2> $O/a2.err || exit $?
timeout -k 10 300 env $ENVB python bench.py --no-cpu-baseline --steps 20 "$@" > $O/b2.json 2> $O/b2.err || exit $?
for f in a1 b a2 b2; do python3 -c "import json;b=json.load(open('$O/$f.json'));print('$f',b['value'],b['ms_per_step'])"; done
