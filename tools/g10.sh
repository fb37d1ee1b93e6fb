# step engine: GPU tests, then step_probe medians (W = 1, 2, 16; step and step5)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py tests/test_wire.py tests/test_stream.py tests/test_c_host.py tests/test_oracle_step.py > gpurun_out/g10_tests.log 2>&1 || exit $?
tail -1 gpurun_out/g10_tests.log
for r in 1 2; do
  for W in 1 2 16; do
    for LEG in step step5; do
      W=$W LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g10.log 2>&1 || exit $?
      python3 - gpurun_out/g10.log $W $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(f"W={sys.argv[2]} {sys.argv[3]} median {statistics.median(ms):.3f} ms/step")
PY
    done
  done
done
