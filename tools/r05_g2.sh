cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/engine_probe.py > gpurun_out/r05_probe.log 2>&1; rc=$?
tail -30 gpurun_out/r05_probe.log; exit $rc
