#!/bin/bash
# One GPU-box session: parity tests, smoke, the default bench line, the multi-GPU rehearsals,
# then rocprofv3 evidence (kernel trace + one PMC pass per counter) of the workloads in PROFILE.
# Stops at the first fault / timeout / abort; a plain test failure (pytest exit 1) still lets the
# bench run. Knobs (environment):
#   TESTS="tests/test_x.py ..."  PYTEST_K="expr"   the GPU tests to run (default: all of -m gpu)
#   SKIP_TESTS=1 SKIP_BENCH=1     skip those steps;  BENCH_ARGS="..." extra bench.py arguments
#   REHEARSE=0                    skip the --gpus 2 threads rehearsal (default on)
#   REHEARSE_TORCHRUN=1 REHEARSE8=1   the torchrun N = 2 and the --gpus 8 c5tl rehearsals
#   AB="tools/ab_engine.py ..."   python scripts run after the bench (A/B drivers), one step each
#   PROFILE="c3mtl c4pq ..."      tools/profile_bench.sh per workload
# (replaces the round-2 gpu_r02.sh and the round-3 one-off g1.sh ... g17.sh, which git history
# keeps as they were run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  rc=$?; if fatal $rc; then exit $rc; fi
  step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
  rc=$?; if fatal $rc; then exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench 600 python -u bench.py ${BENCH_ARGS:-}
  rc=$?; if fatal $rc; then exit $rc; fi
  tail -n 1 gpurun_out/bench.log | wc -c
fi
# launcher-free multi-GPU path, rehearsed with two host threads (two contexts on one GPU)
if [ "${REHEARSE:-1}" = 1 ]; then
  step bench_n2_threads 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu \
    --extra c5v5tl,c4p,cqp --detail-out gpurun_out/bench_n2_detail.json
  rc=$?; if fatal $rc; then exit $rc; fi
fi
# the driver's multi-GPU launch (torchrun, one rank per GPU), rehearsed with two ranks sharing
# the one GPU (gloo for the timing collectives), and BASELINE config 5's 8-GPU share layout with
# eight contexts on the one GPU
if [ "${REHEARSE_TORCHRUN:-0}" = 1 ]; then
  step bench_torchrun_n2 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu \
    --extra c5v5tl --detail-out gpurun_out/bench_torchrun_n2_detail.json
  rc=$?; if fatal $rc; then exit $rc; fi
fi
if [ "${REHEARSE8:-0}" = 1 ]; then
  step bench_c5tl_n8_threads 400 python -u bench.py --gpus 8 --workload c5tl --steps 20 \
    --warmup 5 --no-cpu --extra= --detail-out gpurun_out/bench_c5tl_n8_detail.json
  rc=$?; if fatal $rc; then exit $rc; fi
fi
for A in ${AB:-}; do
  step ab_$(basename $A .py) 300 python -u $A || exit $?
done
for W in ${PROFILE:-}; do
  step prof_$W 400 bash tools/profile_bench.sh $W || exit $?
done
