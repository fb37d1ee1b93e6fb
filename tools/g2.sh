# GPU check of the table ingest: parity tests, the ing legs, a rocprofv3 kernel trace of them
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_ingest.py -m gpu > gpurun_out/g2_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload c2tl --no-cpu --steps 50 --warmup 5 --extra ing,ingu,ingo --detail-out gpurun_out/g2_detail.json > gpurun_out/g2_bench.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g2_prof -o run -- python3 bench.py --workload c2tl --no-cpu --steps 50 --warmup 5 --extra ing --detail-out gpurun_out/g2_detail2.json > gpurun_out/g2_prof.log 2>&1
