#!/bin/bash
# A/B of the lag kernels' groups per lane: default build (4, 16-byte loads) vs tools/lib_vec2 (2,
# 8-byte loads), interleaved, 3 rounds each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in vec4 vec2; do
    if [ $v = vec2 ]; then export HQ_LIB_PATH=tools/lib_vec2/libhipquorum.so; else unset HQ_LIB_PATH; fi
    timeout -k 10 120 python -u bench.py --workload c2l --extra c3l,c5l --no-cpu --steps 200 --warmup 20 > gpurun_out/ab_$v.json 2>/dev/null || exit 7
    echo -n "$v r$r "; python3 -c "
import json,sys; r=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('c2l %.2f us' % r['roofline']['kernel_avg_us'], ' '.join('%s %.2f us' % (e['workload'][:3], e['kernel_avg_us']) for e in r['extra']))"
  done
done
