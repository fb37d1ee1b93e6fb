#!/bin/bash
# Round 6: the late-starting device steps — the step legs with their CPU replay and without it
# (BENCH_STEP_REPLAY=0; the run's other oracle checks kept), alternated. Outputs under $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06l4}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out $O/replay_$i.json > $O/replay_$i.log 2>&1 || exit $?
  BENCH_STEP_REPLAY=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out $O/noreplay_$i.json > $O/noreplay_$i.log 2>&1 || exit $?
done
echo all ok
