#!/bin/bash
# A/B of two builds of libhipquorum.so on the same box: bench legs alternated ROUNDS times,
# default build (A) vs $HQ_B (B, e.g. tools/lib_split/libhipquorum.so). Prints kernel us per leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=${HQ_B:?set HQ_B to the B library}
LEGS=${LEGS:-c2tl}
ROUNDS=${ROUNDS:-3}
HEAD=${HEAD:-c3mtl}
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=$B; fi
    timeout -k 10 120 python3 bench.py --workload $HEAD --extra=$LEGS --no-cpu --steps 400 \
      --warmup 20 ${EXTRA_ARGS:-} > gpurun_out/ab/$v$r.log 2>&1 || exit $?
    python3 - gpurun_out/ab/$v$r.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
legs = [(d["config"]["workload"].split(":")[0], d["roofline"]["kernel_avg_us"])]
legs += [(e["workload"].split(":")[0], e.get("kernel_avg_us") or e.get("ms_per_step")) for e in d["extra"]]
print(sys.argv[2], " ".join(f"{n}={u:.3f}" for n, u in legs if u))
PY
  done
done
