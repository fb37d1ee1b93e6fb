#!/bin/bash
# GPU session: tests, bitmap-tile bench legs, rocprofv3 stats + PMC for c4t / c4ut.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/gpu_tests.log; exit 2; }
tail -n 1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --extra c4,c4t,c4u,c4ut --no-cpu > gpurun_out/bench_c4.log 2>&1 || { tail -n 20 gpurun_out/bench_c4.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_c4.log
PROF="${PROF:-c4t c4ut c4 c4u}" bash tools/prof_only.sh || exit 5
echo session-done
