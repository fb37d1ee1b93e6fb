#!/bin/bash
# Round 6: the engine's static split with reweighted shares (k_engine_reweight). The engine GPU
# tests, the per-workgroup clocks with and without the reweighting (tools/engine_wgprof.py on
# the -DHQ_ENGINE_WGPROF build), then the bench line without extras, reweighted and not, twice
# each, alternated. Outputs under gpurun_out/r06s/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > $O/engine_tests.log 2>&1 || exit $?
WINDOWS=8 HQ_LIB_PATH=tools/lib_engprof/libhipquorum.so timeout -k 10 120 python3 -u tools/engine_wgprof.py > $O/wgprof_rw.log 2>&1 || exit $?
HQ_ENGINE_REWEIGHT=0 WINDOWS=4 HQ_LIB_PATH=tools/lib_engprof/libhipquorum.so timeout -k 10 120 python3 -u tools/engine_wgprof.py > $O/wgprof_uniform.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra= > $O/bench_rw_$i.log 2>&1 || exit $?
  HQ_ENGINE_REWEIGHT=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --extra= > $O/bench_uniform_$i.log 2>&1 || exit $?
done
echo all ok
