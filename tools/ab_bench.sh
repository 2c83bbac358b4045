set -u
O=gpurun_out/ab1; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/a.json 2> $O/a.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --tune ksplit=1 --tune xcd_map=1 > $O/b.json 2> $O/b.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/c.json 2> $O/c.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err
echo PROF $?
