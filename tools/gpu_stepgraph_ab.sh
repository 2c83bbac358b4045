set -u
O=gpurun_out/sg1; mkdir -p $O/db
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/$O/db
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_optim.py tests/test_gpu_matcher.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --phase-timing --no-step-graph > $O/a.json 2> $O/a.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --phase-timing > $O/b.json 2> $O/b.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --phase-timing > $O/c.json 2> $O/c.err || exit $?
echo DONE
