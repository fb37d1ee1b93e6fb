#!/bin/bash
# A/B: fused mixed launches with 1024-thread blocks for every voter count (tools/lib_fb8) vs the
# default (1024 only when every bucket has n <= 5), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in def hf; do
    if [ $v = def ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_$v/libhipquorum.so; fi
    timeout -k 10 200 python -u bench.py --workload c5l --extra c5t --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 7
    echo -n "$v r$r "; python3 -c "
import json; r=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('c5l %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f' % (e['workload'].split(':')[0], e['kernel_avg_us']) for e in r['extra']))"
  done
done
