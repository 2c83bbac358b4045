#!/bin/bash
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6t; mkdir -p $O/db
cp $GRAFT_REPO_ROOT/multimodal-moe_amd/miopen_db/*.txt $O/db/
export MIOPEN_USER_DB_PATH=$O/db
cd $GRAFT_REPO_ROOT
for t in 0 32 16 0 32 16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --eval-steps 0 --tune conv_wg_splits=$t > $O/s$t.json 2> $O/s$t.err || exit $?
  python3 -c "import json;b=json.load(open('$O/s$t.json'));print('splits<=$t',b['value'],b['ms_per_step'])"
done
