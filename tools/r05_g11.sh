# r05k: engine tests, then the default line twice
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05k_engine_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_engine_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/r05_g10.sh
