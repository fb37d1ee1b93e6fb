#!/bin/bash
# Round 6: the balanced engine (per-XCD tile pools, device tickets): the engine tests under it,
# then the headline's engine legs A/B: balanced chunks 4 / 2 / 8 against the static ownership
# (HQ_ENGINE_BALANCE=0). Outputs under gpurun_out/r06i/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
export HQ_ENGINE_WAIT_MS=20000
HQ_ENGINE_BALANCE=1 timeout -k 10 150 python -u -m pytest -v --timeout 60 --timeout-method thread -m gpu tests/test_gpu_engine.py > $O/engine_tests_balanced.log 2>&1 || exit $?
timeout -k 10 150 python -u -m pytest -v --timeout 60 --timeout-method thread -m gpu tests/test_gpu_engine.py > $O/engine_tests.log 2>&1 || exit $?
for V in "1 16" "0 16" "1 8" "1 32" "1 16"; do
  set -- $V
  HQ_ENGINE_BALANCE=$1 HQ_ENGINE_CHUNK=$2 timeout -k 10 130 python -u bench.py --steps 20 --warmup 5 --windows 5 --extra "" --no-cpu --detail-out $O/eng_b$1_c$2.json > $O/eng_b$1_c$2.log 2>&1 || exit $?
  tail -1 $O/eng_b$1_c$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', 'engine', d['engine']['frac'], d['engine']['window_ms'], 'fused', d['fused_window']['frac'], 'signal', d['engine_signal']['median_ms_per_step'], d['engine']['engine_equals_launch_set0'])"
done
echo all ok
