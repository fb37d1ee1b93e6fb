#!/bin/bash
# Round 6: the slot / wait tests (HQ_WAIT_ADAPT added), then the step legs under the adaptive
# and the blocking wait. Outputs under gpurun_out/r06j/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit $?
for P in adapt block; do
  BENCH_STEP_WAIT=$P timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --extra step,step5 --no-extra-parity --detail-out $O/steplegs_$P.json > $O/steplegs_$P.log 2>&1 || exit $?
  python - $O/steplegs_$P.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for r in d["extra"]:
    if r["name"] in ("step", "step5"):
        print(sys.argv[1], r["name"], {k: (v["p50"], v["p99"]) for k, v in r["latency_ms"].items()}, "link", r["link"]["frac"])
PY
done
echo all ok
