#!/bin/bash
# Does a MIOpen user find-db carried between runs make the convolution choice
# (and so the step time) repeatable?  Three bench runs sharing one db dir.
set -u
O=gpurun_out/mdb; mkdir -p $O/db
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/$O/db
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --phase-timing > $O/b$i.json 2> $O/b$i.err || exit $?
  ls -la $O/db > $O/ls$i.txt
done
echo DONE
