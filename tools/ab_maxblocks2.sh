#!/bin/bash
# A/B of the grid cap on the fused mixed launches: default (16384) vs tools/lib_mb4096.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in 16384 4096; do
    if [ $v = 16384 ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_mb$v/libhipquorum.so; fi
    timeout -k 10 200 python -u bench.py --workload c5t --extra c5,c5v5t,c5l --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_mb$v.json 2>gpurun_out/ab_mb$v.err || exit 7
    echo -n "mb$v r$r "; python3 -c "
import json,sys; r=json.loads(open('gpurun_out/ab_mb$v.json').read().strip().splitlines()[-1])
print('c5t %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f' % (e['workload'].split(':')[0], e['kernel_avg_us']) for e in r['extra']))"
  done
done
