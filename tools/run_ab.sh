#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bits.py > gpurun_out/ab_bits.log 2>&1; echo "ab_bits rc=$?"; cat gpurun_out/ab_bits.log
timeout -k 10 300 python -u tools/ab_streams.py > gpurun_out/ab_streams.log 2>&1; echo "ab_streams rc=$?"; cat gpurun_out/ab_streams.log
