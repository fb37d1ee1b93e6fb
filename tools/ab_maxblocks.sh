#!/bin/bash
# A/B of the grid cap (HQ_MAX_BLOCKS, 256-thread units): default 4096 vs tools/lib_mb*, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 4096 8192 16384 32768; do
    if [ $v = 4096 ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_mb$v/libhipquorum.so; fi
    timeout -k 10 200 python -u bench.py --workload c5v5t --extra c2t,c3mt,c5t,c5v5r32t,c5l,c4u,cq --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_mb$v.json 2>gpurun_out/ab_mb$v.err || exit 7
    echo -n "mb$v r$r "; python3 -c "
import json,sys; r=json.loads(open('gpurun_out/ab_mb$v.json').read().strip().splitlines()[-1])
print('c5v5t %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f' % (e['workload'].split(':')[0], e['kernel_avg_us']) for e in r['extra']))"
  done
done
