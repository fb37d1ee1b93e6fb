#!/bin/bash
# Round 6: the late-starting device steps — the step legs with their CPU replay, the runtime's
# large pageable copies staged (GPU_PINNED_MIN_XFER_SIZE raised: no pin-in-place of the caller's
# pages) against its default, alternated. Outputs under $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06l5}
mkdir -p $O
for i in 1 2; do
  GPU_PINNED_MIN_XFER_SIZE=1000000 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out $O/staged_$i.json > $O/staged_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out $O/default_$i.json > $O/default_$i.log 2>&1 || exit $?
done
echo all ok
