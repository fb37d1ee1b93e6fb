# binned-ingest phase timings, parity tests, ing legs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/binprof > gpurun_out/g3_binprof.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_table.py -m gpu > gpurun_out/g3_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload c2tl --no-cpu --steps 50 --warmup 5 --extra ing,ingu --detail-out gpurun_out/g3_detail.json > gpurun_out/g3_bench.log 2>&1
