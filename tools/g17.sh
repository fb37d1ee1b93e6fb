# step engine: every worker-level GPU test, step_probe medians (W = 1, 2, 16), step5 timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py tests/test_wire.py tests/test_stream.py tests/test_c_host.py tests/test_oracle_step.py > gpurun_out/g17_tests.log 2>&1 || exit $?
tail -1 gpurun_out/g17_tests.log
for r in 1 2; do
  for W in 1 2 16; do
    for LEG in step step5; do
      W=$W LEG=$LEG STEPS=10 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g17.log 2>&1 || exit $?
      python3 - gpurun_out/g17.log $W $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(f"W={sys.argv[2]} {sys.argv[3]} median {statistics.median(ms):.3f} ms/step")
PY
    done
  done
done
for W in 1 16; do
  LEG=step5 W=$W STEPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/g17_w$W -o run -- python3 tools/step_probe.py > gpurun_out/g17_w$W.log 2>&1 || exit $?
  INPUT_MB=38.5 python3 tools/step_timeline.py gpurun_out/g17_w$W 4 $W > gpurun_out/g17_timeline_w$W.txt 2>&1
  cat gpurun_out/g17_timeline_w$W.txt
done
