#!/bin/bash
# A/B of the threaded event encoder: the default build (persistent task pool) against
# tools/lib_encspawn (threads spawned per call), alternated ROUNDS times on one box: the encode
# probe (tools/enc_probe.py) and the step5 leg (device-only and end to end, no CPU replay).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=${ROUNDS:-2}
O=gpurun_out/ab_encode
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in default encspawn; do
    if [ $v = default ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_$v/libhipquorum.so; fi
    echo "== $v round $r"
    timeout -k 10 120 python3 tools/enc_probe.py || exit $?
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --extra step5 --no-cpu \
      --detail-out $O/$v$r.json > $O/$v$r.log 2>&1 || exit $?
    python3 - $O/$v$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ex = d["extra"]
r = [x for x in ex if x.get("name") == "step5"][0] if isinstance(ex, list) else ex["step5"]
print("step5 medians ms:", {k: round(v["median"], 3) for k, v in r["ms_per_step_detail"].items()},
      "parity/modes", r.get("modes_agree"))
PY
  done
done
