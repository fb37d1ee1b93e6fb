#!/bin/bash
# GPU session: parity tests (new reference scenarios), the stream-layout floor experiment, the
# new bench legs (c4u, ingo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -n 30 gpurun_out/gpu_tests.log; exit 2; }
tail -n 2 gpurun_out/gpu_tests.log
timeout -k 10 120 ./tools/kexp5 > gpurun_out/kexp5.log 2>&1 || { tail gpurun_out/kexp5.log; exit 3; }
cat gpurun_out/kexp5.log
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu --extra c4,c4u,ing,ingo > gpurun_out/bench_legs.log 2>&1 || { tail -n 20 gpurun_out/bench_legs.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_legs.log
echo session-done
