#!/bin/bash
# GPU session: node-scale 5-voter legs (8M x 5 per GPU, mask and u32 ring, tiles) in the bench,
# then rocprofv3 stats + FETCH/WRITE PMC for them and for the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --extra c3mt,c5v5t,c5v5r32t,c5t > gpurun_out/bench_v5.log 2>&1 || { tail -n 20 gpurun_out/bench_v5.log; exit 4; }
python3 tools/summarize_bench.py gpurun_out/bench_v5.log
PROF="${PROF:-c5v5t c5v5r32t c2t}" bash tools/prof_only.sh || exit 5
echo session-done
