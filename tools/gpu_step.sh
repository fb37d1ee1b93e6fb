set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1
rc=$?
tail -5 gpurun_out/engine_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --extra "" --no-cpu > gpurun_out/bench_engine1.log 2> gpurun_out/bench_engine1.err
rc=$?
tail -3 gpurun_out/bench_engine1.err
exit $rc
