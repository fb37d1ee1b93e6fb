#!/bin/bash
# Round 6: the late-starting device steps inside the bench. The step legs alone
# (--extra step,step5), with the CPU replay between the device steps and without it
# (--no-cpu), alternated. Outputs under gpurun_out/r06l2/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06l2}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out $O/cpu_$i.json > $O/cpu_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-cpu --detail-out $O/nocpu_$i.json > $O/nocpu_$i.log 2>&1 || exit $?
done
echo all ok
