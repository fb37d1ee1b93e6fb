#!/bin/bash
# multi-ctx ReadIndex: pair kernel parity (readindex + worker tests), then an interleaved A/B of
# the rim leg with HQ_RI_PAIRS=1 (default) / 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_readindex_multi.py tests/test_gpu_worker.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rim_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/rim_tests.log; exit 2; }
tail -n 1 gpurun_out/rim_tests.log
for r in 1 2 3; do
  for v in 1 0; do
    HQ_RI_PAIRS=$v timeout -k 10 200 python -u bench.py --workload c2t --extra rim --no-cpu --steps 200 --warmup 20 > gpurun_out/rim_$v.json 2>gpurun_out/rim_$v.err || exit 7
    echo -n "pairs=$v r$r "; python3 -c "
import json; r=json.loads(open('gpurun_out/rim_$v.json').read().strip().splitlines()[-1])
e=[x for x in r['extra'] if x['workload'].startswith('rim')][0]; print('rim %.2f us  %.3g releases/s  frac %.3f' % (e['kernel_avg_us'], e['value'], e['roofline_frac']))"
  done
done
