# chunk split A/B (equal, geometric 0.84 / 0.70, 8 chunks at 0.84): step_probe medians, one worker
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
HQ_LIB_PATH=tools/lib_split8c84/libhipquorum.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_worker.py -k "chunked" > gpurun_out/g13_tests.log 2>&1 || exit $?
tail -1 gpurun_out/g13_tests.log
for r in 1 2 3; do
for v in default stepsplit84 stepsplit70 split8c84; do
  if [ $v = default ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=tools/lib_$v/libhipquorum.so; fi
  for LEG in step step5; do
    W=1 LEG=$LEG STEPS=10 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g13.log 2>&1 || exit $?
    python3 - gpurun_out/g13.log $LEG $v <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(f"{sys.argv[3]} W=1 {sys.argv[2]} median {statistics.median(ms):.3f} ms/step")
PY
  done
done
done
