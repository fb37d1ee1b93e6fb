#!/bin/bash
# Round 6: pass A with 2 pending-read slots per group (scratch 96 instead of 336 B per lane) against
# the product build: step5 W = 1 kernel traces. Outputs gpurun_out/r06p/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
for L in base dreads2; do
  if [ $L = base ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_$L/libhipquorum.so; fi
  LEG=step5 SLOTS=1 S16=1 W=1 STEPS=8 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$L -o run -- python3 tools/step_probe.py > $O/prof_$L.log 2>&1 || exit $?
done
echo all ok
