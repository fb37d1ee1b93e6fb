cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_engine_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/r05_engine_tests2.log; [ $rc -ne 0 ] && exit $rc
AB_ONLY=engine,signal,fused,launches timeout -k 10 300 python -u tools/ab_engine.py > gpurun_out/r05_ab_engine2.log 2>&1 || exit $?
tail -5 gpurun_out/r05_ab_engine2.log
for T in 16 14 12; do
  BENCH_HQ_ENCODE_THREADS=$T timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --extra step,step5 --detail-out gpurun_out/r05_steplegs_t$T.json > gpurun_out/r05_steplegs_t$T.log 2>&1 || exit $?
  echo "T=$T done"
done
