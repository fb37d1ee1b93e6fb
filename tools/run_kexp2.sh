#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/kexp2
timeout -k 10 120 ./tools/kexp2 > gpurun_out/kexp2/plain.log 2>&1 || exit $?
cat gpurun_out/kexp2/plain.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kexp2/prof -o k -- ./tools/kexp2 > gpurun_out/kexp2/prof.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/kexp2/prof/k_kernel_stats.csv
