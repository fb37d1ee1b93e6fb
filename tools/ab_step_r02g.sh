mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py tests/test_wire.py tests/test_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/worker_tests.log 2>&1; rc=$?; tail -2 gpurun_out/worker_tests.log; [ $rc -ne 0 ] && exit $rc
for B in prev sw3 sw4; do echo "== A=current B=$B"; HQ_B=tools/lib_$B/libhipquorum.so ROUNDS=1 bash tools/ab_step.sh || exit $?; done
