# device timelines of the step engine, one worker against 16 (rocprofv3 kernel + copy traces)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for W in 1 16; do
  LEG=step5 W=$W STEPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/g5_w$W -o run -- python3 tools/step_probe.py > gpurun_out/g5_w$W.log 2>&1 || exit $?
  head -1 gpurun_out/g5_w$W/run_memory_copy_trace.csv >> gpurun_out/g5_w$W.log
  python3 tools/step_timeline.py gpurun_out/g5_w$W 4 $W > gpurun_out/g5_timeline_w$W.txt 2>&1 || exit $?
done
