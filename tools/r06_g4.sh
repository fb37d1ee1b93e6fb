#!/bin/bash
# Round 6: the wire feeds' worker tests (attached decode counting per handle), then the step legs
# under each wait policy (hq_worker_set_wait; device clocks on) with the link block, the engine
# sharing leg, and the wire leg alone. Outputs under gpurun_out/r06d/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "wire" > $O/wire_tests.log 2>&1 || exit $?
for P in block sleep:50:20 spin; do
  n=${P%%:*}
  BENCH_STEP_WAIT=$P timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --extra step,step5 --no-extra-parity --detail-out $O/steplegs_$n.json > $O/steplegs_$n.log 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra share --no-extra-parity --no-cpu --detail-out $O/share.json > $O/share.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --extra wire --no-extra-parity --no-cpu --detail-out $O/wire.json > $O/wire.log 2>&1 || exit $?
echo all ok
