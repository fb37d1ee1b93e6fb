#!/bin/bash
# A/B of library builds on the same box: for the default build and each variant in $VARIANTS
# (tools/lib_<v>/libhipquorum.so, the Makefile's variant targets), the bench legs $LEGS, ROUNDS
# times alternated; prints each leg's kernel time per launch (us) and roofline fraction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LEGS=${LEGS:?set LEGS}
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out/ab_legs
for r in $(seq 1 $ROUNDS); do
  for v in default $VARIANTS; do
    if [ $v = default ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_$v/libhipquorum.so; fi
    timeout -k 10 200 python3 bench.py --workload c2tl --extra $LEGS --no-cpu --steps ${STEPS:-200} \
      --warmup 20 --detail-out gpurun_out/ab_legs/$v$r.json > gpurun_out/ab_legs/$v$r.log 2>&1 || exit $?
    python3 - gpurun_out/ab_legs/$v$r.log $v <<'PY'
import json, sys
out = []
for line in open(sys.argv[1]):
    if line.startswith("extra "):
        d = json.loads(line[6:])
        out.append(f"{d['name']}={d.get('kernel_avg_us', 0):.3f}us/{d.get('roofline_frac', 0):.4f}")
print(sys.argv[2], " ".join(out))
PY
  done
done
