#!/bin/bash
# GPU session: parity tests -> smoke -> bench (all extras) -> 2-rank rehearsal of the N>1 path on
# this 1-GPU box (both ranks on GPU 0, gloo timing collectives) -> rocprofv3 for $PROF workloads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_round3.sh || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 200 --warmup 20 --no-cpu > gpurun_out/bench_n2.log 2>&1 \
  || { tail -n 30 gpurun_out/bench_n2.log; exit 6; }
python3 tools/summarize_bench.py gpurun_out/bench_n2.log
echo round4-done
