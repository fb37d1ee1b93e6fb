#!/bin/bash
# GPU session: tests, then the leader-row tile legs next to their HQ_LAYOUT_TILES twins, profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/gpu_tests.log; exit 2; }
tail -n 1 gpurun_out/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload c2tl --no-cpu --extra c2t,c3mt,c3mtl,c5v5t,c5v5tl,c5t,c5tl > gpurun_out/bench_lead_$i.log 2>&1 || { tail -n 20 gpurun_out/bench_lead_$i.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_lead_$i.log
done
PROF="${PROF:-c2tl c5v5tl c5tl}" bash tools/prof_only.sh || exit 5
echo session-done
