#!/bin/bash
# A/B of the commit kernels' block size: default build (1024-thread blocks where the kernel fits
# 64 VGPRs) vs tools/lib_b512 (512 everywhere), interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in big b512; do
    if [ $v = b512 ]; then export HQ_LIB_PATH=tools/lib_b512/libhipquorum.so; else unset HQ_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --workload c2 --extra c2l,c3m,c3l,c3,c5 --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_$v.json 2>/dev/null || exit 7
    echo -n "$v r$r "; python3 -c "
import json,sys; r=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('c2 %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f us' % (e['workload'][:4], e['kernel_avg_us']) for e in r['extra']))"
  done
done
