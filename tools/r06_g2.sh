#!/bin/bash
# Round 6: the slot / 2-byte / wait / wire forms' GPU tests (a test failure does not stop the
# session), then the wire legs. Outputs under gpurun_out/r06c/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_slots.py > $O/slots_tests.log 2>&1; ok
timeout -k 10 480 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "sized16 or compact or regrow or jobs or wire" > $O/worker_tests.log 2>&1; ok
timeout -k 10 330 python -u bench.py --steps 20 --warmup 5 --extra wire,wire_step --no-extra-parity --detail-out $O/wire_detail.json > $O/wire_bench.log 2>&1; ok
echo all ok
