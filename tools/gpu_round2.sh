#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench.log
for W in c2 c3m; do bash tools/profile_bench.sh $W || exit $?; done
timeout -k 10 200 ./tools/kexp > gpurun_out/kexp.log 2>&1; tail -n 40 gpurun_out/kexp.log
