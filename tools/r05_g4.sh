cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/enc_probe.py > gpurun_out/r05_enc_probe.log 2>&1; rc=$?
cat gpurun_out/r05_enc_probe.log | tail -12; exit $rc
