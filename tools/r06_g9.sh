#!/bin/bash
# Round 6: pass A with the stream read in place (zero copy) against the stream copied to the
# device first (HQ_STEP_ZERO_COPY=0), step5 W = 1, kernel traces. Outputs gpurun_out/r06l/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
for Z in 1 0; do
  HQ_STEP_ZERO_COPY=$Z LEG=step5 SLOTS=1 S16=1 W=1 STEPS=8 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof_z$Z -o run -- python3 tools/step_probe.py > $O/prof_z$Z.log 2>&1 || exit $?
done
echo all ok
