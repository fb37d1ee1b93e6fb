#!/bin/bash
# bitmap kernels: parity (every bitmap test), then the c4 / c4t / c4u / c4ut / cq legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "bits or bitmap or vote or readindex or check_quorum or worker" --timeout 120 --timeout-method thread > gpurun_out/bits_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/bits_tests.log; exit 2; }
tail -n 1 gpurun_out/bits_tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c2t --extra c4,c4t,c4u,c4ut,cq --no-cpu > gpurun_out/bench_bits.log 2>&1 || { tail -n 20 gpurun_out/bench_bits.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_bits.log | grep -v headline
done
