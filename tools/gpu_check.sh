#!/bin/bash
# Validation session: parity tests, smoke, default bench, stream-overlap experiment.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 30 gpurun_out/gpu_tests.log; exit 2; }
tail -n 3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -n 20 gpurun_out/bench.log; exit 4; }
tail -c 600 gpurun_out/bench.log
if [ -n "${AB:-}" ]; then timeout -k 10 300 python -u tools/ab_streams.py > gpurun_out/ab_streams.log 2>&1 || { tail gpurun_out/ab_streams.log; exit 5; }; cat gpurun_out/ab_streams.log; fi
echo session-done
