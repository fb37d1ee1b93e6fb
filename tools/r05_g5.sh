# r05d: the step legs with the device split (GPU event time vs the host's wait) per step
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_leg.py tests/test_gpu_worker.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05d_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-cpu --detail-out gpurun_out/r05d_detail.json > gpurun_out/r05d_bench.log 2>&1 || exit $?
tail -c 400 gpurun_out/r05d_bench.log; echo; echo done
