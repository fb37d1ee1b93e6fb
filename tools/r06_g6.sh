#!/bin/bash
# Round 6: the device step (step5, slots + 2-byte size words) under rocprofv3 kernel trace for
# W = 1 and 16, the host phases of each jobs call (HQ_STEP_JOBS_TRACE), and the headline's
# kernel trace with the engine legs. Outputs under gpurun_out/r06h/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
for W in 1 16; do
  LEG=step5 SLOTS=1 S16=1 W=$W STEPS=8 HQ_STEP_JOBS_TRACE=1 timeout -k 10 200 python -u tools/step_probe.py > $O/probe_w$W.log 2>&1 || exit $?
  LEG=step5 SLOTS=1 S16=1 W=$W STEPS=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_w$W -o run -- python3 tools/step_probe.py > $O/prof_w$W.log 2>&1 || exit $?
done
echo all ok
