#!/bin/bash
# GPU session: parity, the same-box layout A/B (kexp6), the column / tile legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/gpu_tests.log; exit 2; }
tail -n 2 gpurun_out/gpu_tests.log
timeout -k 10 200 ./tools/kexp7 > gpurun_out/kexp7.log 2>&1 || { tail gpurun_out/kexp7.log; exit 3; }
cat gpurun_out/kexp7.log
timeout -k 10 400 python -u bench.py --workload c2t --steps 400 --no-cpu --extra ${EXTRA:-c2,c2l,c3m,c3mt,c3r32,c3r32t,c5,c5t} > gpurun_out/bench_tiles.log 2>&1 || { tail -n 20 gpurun_out/bench_tiles.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_tiles.log
echo session-done
