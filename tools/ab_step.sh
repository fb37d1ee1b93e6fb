#!/bin/bash
# A/B of two builds on the device step engine: tools/step_probe.py (1 M groups, event stream)
# alternated ROUNDS times, default build (A) vs $HQ_B (B); prints the median of the last steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=${HQ_B:?set HQ_B to the B library}
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out/abs
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=$B; fi
    for W in ${WS:-1 16}; do
      for LEG in ${LEGS:-step step5}; do
        W=$W LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/abs/$v$r.$W.$LEG.log 2>&1 || exit $?
        python3 - gpurun_out/abs/$v$r.$W.$LEG.log $v $W $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(sys.argv[2], f"W={sys.argv[3]} {sys.argv[4]} median {statistics.median(ms):.2f} ms/step")
PY
      done
    done
  done
done
