# r05e: the device step's tests, then kernel timelines of the step5 device step for each
# environment setting in VARS (space-separated NAME=VALUE, one run each) and worker count in WS
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05e}
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_step_leg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for V in ${VARS:-HQ_STEP_SPEC_READY=1}; do
for W in ${WS:-1 16}; do
  n=${T}_${V//=/}_w$W
  ( export $V LEG=step5 W=$W STEPS=6; timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/$n -o run -- python3 tools/step_probe.py > gpurun_out/${n}.log 2>&1 ) || { tail gpurun_out/${n}.log; exit 4; }
  python3 tools/step_timeline.py gpurun_out/$n 6 $W > gpurun_out/${n}_timeline.txt 2>&1 || exit 5
  echo "== $V W=$W"; grep "step 5" gpurun_out/${n}.log; head -12 gpurun_out/${n}_timeline.txt
done
done
echo done
