#!/bin/bash
# Round 6: run members taken at once on the device (take_run): every GPU test, the step legs, and
# the step5 kernel trace. Outputs under gpurun_out/r06n/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_worker.py -k consecutive > $O/runs_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-extra-parity --detail-out $O/steplegs.json > $O/steplegs.log 2>&1 || exit $?
LEG=step5 SLOTS=1 S16=1 W=1 STEPS=8 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_w1 -o run -- python3 tools/step_probe.py > $O/prof_w1.log 2>&1 || exit $?
echo all ok
