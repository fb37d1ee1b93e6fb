# A/B: pass A's waves per SIMD (HQ_STEP_WAVES builds in tools/lib_waves/) on the step5 device step
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for L in base w3 w4; do
  if [ $L = base ]; then unset HQ_LIB_PATH; else export HQ_LIB_PATH=$PWD/tools/lib_waves/libhipquorum_$L.so; fi
  for W in 1 16; do
    LEG=step5 W=$W STEPS=8 timeout -k 10 200 python3 -u tools/step_probe.py > gpurun_out/abw_${L}_$W.log 2>&1 || { tail -3 gpurun_out/abw_${L}_$W.log; exit 3; }
    python3 -c "
import re,statistics
t=[float(m.group(1)) for m in re.finditer(r'max device ([0-9.]+) ms', open('gpurun_out/abw_${L}_$W.log').read())][2:]
w=[float(m.group(1)) for m in re.finditer(r'step \d+: ([0-9.]+) ms', open('gpurun_out/abw_${L}_$W.log').read())][2:]
print('$L W=$W device median %.3f ms wall median %.3f' % (statistics.median(t), statistics.median(w)))"
  done
done
done
