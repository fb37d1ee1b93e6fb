#!/bin/bash
# GPU session: tests, then the fused (mixed-membership) legs twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/gpu_tests.log; exit 2; }
tail -n 1 gpurun_out/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload c5tl --no-cpu --extra c5t,c5,c5l,c5ll,c2tl > gpurun_out/bench_fused_$i.log 2>&1 || { tail -n 20 gpurun_out/bench_fused_$i.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_fused_$i.log
done
echo session-done
