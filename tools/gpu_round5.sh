#!/bin/bash
# GPU session: tests + smoke + bench (gpu_round3.sh), then a 3-rank rehearsal on the one GPU
# (world divisible by 3: the mixed-membership legs are skipped, the headline line still prints).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_round3.sh || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --gpus 3 --steps 100 --warmup 10 --no-cpu --extra c5,c2l,e2e > gpurun_out/bench_n3.log 2>&1 \
  || { tail -n 30 gpurun_out/bench_n3.log; exit 6; }
python3 tools/summarize_bench.py gpurun_out/bench_n3.log
echo round5-done
