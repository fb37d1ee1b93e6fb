#!/bin/bash
# GPU session: parity tests -> bench -> 2-rank rehearsal of the N>1 path on this 1-GPU box
# (both ranks on GPU 0, gloo for the timing collectives) -> rocprofv3 for $PROF workloads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -n 20 gpurun_out/bench.log; exit 3; }
tail -n 1 gpurun_out/bench.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 200 --warmup 20 --no-cpu --extra '' > gpurun_out/bench_n2.log 2>&1 \
  || { tail -n 30 gpurun_out/bench_n2.log; exit 5; }
tail -n 1 gpurun_out/bench_n2.log
for W in ${PROF:-}; do bash tools/profile_bench.sh $W > gpurun_out/profile_$W.log 2>&1 || { tail gpurun_out/profile_$W.log; exit 4; }; done
echo session-done
