#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/prof_kexp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kexp -o kexp -- ./tools/kexp > gpurun_out/prof_kexp/stdout.log 2>&1
rc=$?; echo rc=$rc
find gpurun_out/prof_kexp -name "*stats*" | head
f=$(find gpurun_out/prof_kexp -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -40
exit $rc
