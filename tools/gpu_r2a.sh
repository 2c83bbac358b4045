set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2a; mkdir -p $O; cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "PYTEST $rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "BENCH $rc"; cat $O/bench.json
exit $rc
