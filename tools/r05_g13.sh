# r05o: the device step's tests, its host phases (HQ_STEP_JOBS_TRACE) at W = 1 and 16, then the
# driver's line with the step legs
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05o}
timeout -k 10 400 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_step_leg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for W in 1 16; do
  HQ_STEP_JOBS_TRACE=1 LEG=step5 W=$W STEPS=10 timeout -k 10 200 python3 tools/step_probe.py > gpurun_out/${T}_trace_w$W.log 2>&1 || exit 4
  tail -4 gpurun_out/${T}_trace_w$W.log
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out gpurun_out/${T}_detail.json > gpurun_out/${T}_bench.log 2>&1 || exit 5
python3 - gpurun_out/${T}_detail.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline %.4g frac %.4f engine %.4f launch %.4f" % (d["value"], d["roofline"]["frac"], d["engine"]["frac"], d["launch_per_step"]["frac"]))
for x in d.get("extra", []):
    if isinstance(x, dict) and "latency_ms" in x:
        print(x.get("name"), {k: v["p50"] for k, v in x["latency_ms"].items()}, "e2e", {k: round(v / 1e9, 3) for k, v in x["end_to_end"].items()}, "vs replay", {k: round(v, 2) for k, v in x.get("vs_cpu_replay_end_to_end", {}).items()}, "parity", x.get("parity_committed"))
PY
