# A/B: the tree's library against tools/lib_ab/libhipquorum_base.so (the last commit's device step)
# on the step5 device step, W = 1 and 16, two alternated rounds
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for L in base new; do
  if [ $L = base ]; then export HQ_LIB_PATH=$PWD/tools/lib_ab/libhipquorum_base.so; else unset HQ_LIB_PATH; fi
  for W in 1 16; do
    LEG=${LEG:-step5} W=$W STEPS=8 timeout -k 10 200 python3 -u tools/step_probe.py > gpurun_out/abl_${L}_$W.log 2>&1 || { tail -3 gpurun_out/abl_${L}_$W.log; exit 3; }
    python3 -c "
import re,statistics
s=open('gpurun_out/abl_${L}_$W.log').read()
t=[float(m.group(1)) for m in re.finditer(r'max device ([0-9.]+) ms', s)][2:]
w=[float(m.group(1)) for m in re.finditer(r'step \d+: ([0-9.]+) ms', s)][2:]
print('$L W=$W device median %.3f ms wall median %.3f' % (statistics.median(t), statistics.median(w)))"
  done
done
done
