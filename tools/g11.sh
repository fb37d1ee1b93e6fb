# step engine after k_ready_out: worker GPU tests, step_probe medians, step5 timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "chunked or rejected" > gpurun_out/g11_tests.log 2>&1 || exit $?
tail -1 gpurun_out/g11_tests.log
for W in 1 2 16; do
  for LEG in step step5; do
    W=$W LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g11.log 2>&1 || exit $?
    python3 - gpurun_out/g11.log $W $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(f"W={sys.argv[2]} {sys.argv[3]} median {statistics.median(ms):.3f} ms/step")
PY
  done
done
LEG=step5 W=1 STEPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/g11_w1 -o run -- python3 tools/step_probe.py > gpurun_out/g11_w1.log 2>&1 || exit $?
INPUT_MB=38.5 python3 tools/step_timeline.py gpurun_out/g11_w1 4 1 > gpurun_out/g11_timeline_w1.txt 2>&1
cat gpurun_out/g11_timeline_w1.txt
