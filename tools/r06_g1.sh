#!/bin/bash
# Round 6, first box: the new device-step forms' tests, then the step5 device step with and
# without them (tools/step_probe.py medians). Outputs under gpurun_out/r06a/. A test failure
# (pytest rc 1) does not stop the session; anything else does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python -u tools/dbg_regrow.py > $O/dbg_regrow.log 2>&1; ok
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_slots.py > $O/slots_tests.log 2>&1; ok
timeout -k 10 900 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "sized16 or compact or regrow or jobs or wire" > $O/worker_tests.log 2>&1; ok
for W in 1 16; do
  for V in "base:COMPACT=1" "s16:COMPACT=1 S16=1" "slots:SLOTS=1 S16=1"; do
    n=${V%%:*}; envs=${V#*:}
    env $envs LEG=step5 W=$W STEPS=12 timeout -k 10 300 python -u tools/step_probe.py > $O/probe_${n}_w$W.log 2>&1 || exit $?
  done
done
echo all ok
