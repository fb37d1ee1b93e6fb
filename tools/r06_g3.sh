#!/bin/bash
# Round 6: the step legs under each wait policy (p50 / p99 and the wait's clocks), then the
# GPU-sharing leg. Outputs under gpurun_out/r06d/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
for P in block sleep:50:20 spin; do
  n=${P%%:*}
  BENCH_STEP_WAIT=$P timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-extra-parity --detail-out $O/steplegs_$n.json > $O/steplegs_$n.log 2>&1 || exit $?
done
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --extra share --no-extra-parity --no-cpu --detail-out $O/share.json > $O/share.log 2>&1 || exit $?
echo all ok
