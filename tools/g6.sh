# device step engine: its GPU tests, then the step legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py tests/test_wire.py tests/test_stream.py tests/test_c_host.py tests/test_oracle_step.py > gpurun_out/g6_tests.log 2>&1 && \
for W in 1 16; do LEG=step5 W=$W STEPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/g6_w$W -o run -- python3 tools/step_probe.py > gpurun_out/g6_w$W.log 2>&1 || exit $?; done && \
LISTS=1 LEG=step W=1 STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g6_step_w1.log 2>&1
