#!/bin/bash
# rocprofv3 kernel stats of tools/kexp6 (per-kernel durations behind its event timings)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/prof_kexp6
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kexp6 -o k -- ./tools/kexp6 > gpurun_out/prof_kexp6/stdout.log 2>&1 || exit $?
cat gpurun_out/prof_kexp6/stdout.log
f=$(find gpurun_out/prof_kexp6 -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
