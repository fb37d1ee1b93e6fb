#!/bin/bash
# GPU session: tests, smoke, default bench, rocprofv3 stats + PMC of the given legs.
# tiled and column legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/gpu_tests.log; exit 2; }
tail -n 1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -n 20 gpurun_out/bench.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench.log
PROF="${PROF:-c2t rim}" bash tools/prof_only.sh || exit 5
echo session-done
