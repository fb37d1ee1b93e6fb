set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "rejected_steps or input_errors" > gpurun_out/g9_tests.log 2>&1
