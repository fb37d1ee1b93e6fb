set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_planes_cq.py tests/test_cq_planes.py tests/test_bits3.py -m gpu > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --extra c4p,cqp,c4pq --detail-out gpurun_out/g1_detail.json > gpurun_out/g1_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g1_prof -o run -- python3 bench.py --steps 100 --warmup 10 --extra c4pq --detail-out gpurun_out/g1_detail2.json > gpurun_out/g1_prof.log 2>&1
