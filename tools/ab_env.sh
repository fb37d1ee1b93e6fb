#!/bin/bash
# The device step engine (tools/step_probe.py) with and without an environment setting
# (ENV_B="NAME=value"), alternated ROUNDS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out/abe
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    for W in ${WS:-1 16}; do
      for LEG in ${LEGS:-step step5}; do
        if [ $v = A ]; then
          W=$W LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/abe/$v$r.$W.$LEG.log 2>&1 || exit $?
        else
          env $ENV_B W=$W LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/abe/$v$r.$W.$LEG.log 2>&1 || exit $?
        fi
        python3 - gpurun_out/abe/$v$r.$W.$LEG.log $v $W $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(sys.argv[2], f"W={sys.argv[3]} {sys.argv[4]} median {statistics.median(ms):.2f} ms/step")
PY
      done
    done
  done
done
