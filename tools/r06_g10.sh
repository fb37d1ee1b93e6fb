#!/bin/bash
# Round 6: pass A zero copy vs copied (r06_g9), the encode placement probe (r06_g8), then the step
# legs twice with the device's start and end stamps (the span of each step). gpurun_out/r06m/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
bash tools/r06_g9.sh > $O/g9.log 2>&1 || exit $?
bash tools/r06_g8.sh > $O/g8.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu --extra step,step5 --no-extra-parity --detail-out $O/steplegs_$k.json > $O/steplegs_$k.log 2>&1 || exit $?
done
echo all ok
