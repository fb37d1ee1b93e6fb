#!/bin/bash
# A/B of 1024-thread blocks for the n = 5 ring-gather commit kernels (default build) against
# 512 everywhere (tools/lib_b512), interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in big b512; do
    if [ $v = b512 ]; then export HQ_LIB_PATH=tools/lib_b512/libhipquorum.so; else unset HQ_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --workload c3 --extra c3r32 --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_$v.json 2>/dev/null || exit 7
    echo -n "$v r$r "; python3 -c "
import json,sys; r=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('c3 %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f us' % (e['workload'][:5], e['kernel_avg_us']) for e in r['extra']))"
  done
done
