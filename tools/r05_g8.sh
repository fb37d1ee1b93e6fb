# r05h: device-step and encoder tests, then the step legs of the bench
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05h}
timeout -k 10 400 python -u -m pytest tests/test_stream.py tests/test_gpu_worker.py tests/test_gpu_step_leg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out gpurun_out/${T}_detail.json > gpurun_out/${T}_bench.log 2>&1 || exit $?
tail -c 900 gpurun_out/${T}_bench.log; echo; echo done
