cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_engine_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_engine_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_engine.py > gpurun_out/r05_ab_engine.log 2>&1
rc=$?; tail -25 gpurun_out/r05_ab_engine.log; echo "ab rc=$rc"; exit $rc
