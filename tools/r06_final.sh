#!/bin/bash
# One GPU-box validation of the tree (round 6): every GPU test, smoke, the driver's bench command,
# the --gpus 2 threads and torchrun rehearsals; each step under its own time limit, stopping at
# the first failure. Outputs under gpurun_out/r06final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 380 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
T0=$(date +%s); timeout -k 10 380 python -u bench.py --steps 20 --warmup 5 --detail-out $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit $?; echo "bench wall $(( $(date +%s) - T0 )) s" > $O/bench_wall.txt
timeout -k 10 140 python -u bench.py --gpus 2 --steps 20 --warmup 5 --extra= --detail-out $O/n2_detail.json > $O/bench_n2_threads.log 2>&1 || exit $?
timeout -k 10 140 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --extra= --detail-out $O/tr2_detail.json > $O/bench_torchrun_n2.log 2>&1 || exit $?
echo all ok
