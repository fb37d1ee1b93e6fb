# 16 step workers with 4 (the box default) and 16 hardware queues per process
cd $GRAFT_REPO_ROOT
for q in 4 16 4 16; do
  for LEG in step step5; do
    GPU_MAX_HW_QUEUES=$q W=16 LEG=$LEG STEPS=8 timeout -k 10 120 python3 tools/step_probe.py > gpurun_out/g8.log 2>&1 || exit $?
    python3 - gpurun_out/g8.log $q $LEG <<'PY'
import re, statistics, sys
ms = [float(m.group(1)) for m in re.finditer(r"step [3-9]: ([0-9.]+) ms", open(sys.argv[1]).read())]
print(f"HW queues {sys.argv[2]} W=16 {sys.argv[3]} median {statistics.median(ms):.2f} ms/step")
PY
  done
done
