#!/bin/bash
# GPU session: parity tests -> bench (headline + extras) -> rocprofv3 evidence for $PROF workloads.
# Stops at the first fault / abort / timeout; plain test failures still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -n 20 gpurun_out/bench.log; exit 3; }
tail -n 1 gpurun_out/bench.log
for W in ${PROF:-c2}; do bash tools/profile_bench.sh $W > gpurun_out/profile_$W.log 2>&1 || { tail gpurun_out/profile_$W.log; exit 4; }; done
echo session-done
