cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
PROBE_QUIET=1 PROBE_STEPS=37 timeout -k 10 60 python -u tools/engine_probe.py > gpurun_out/r05_probe_fast.log 2>&1; rc=$?
tail -8 gpurun_out/r05_probe_fast.log
PROBE_QUIET=1 PROBE_STEPS=37 PROBE_G=100000 timeout -k 10 60 python -u tools/engine_probe.py > gpurun_out/r05_probe_fast2.log 2>&1; rc2=$?
tail -8 gpurun_out/r05_probe_fast2.log; exit $((rc+rc2))
