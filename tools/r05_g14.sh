# r05t: step5 device-step timelines with compact ReadyToReads, the product library against a
# build whose k_step_lite skips its ReadyToRead stores (timing probe)
# (the nostore / slots libraries are builds of profiles/r05n/device_step_probes.patch)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05t}
for L in ${LIBS:-base nostore}; do
for W in 1 16; do
  n=${T}_${L}_w$W
  case $L in nostore) LP=tools/lib_litenostore/libhipquorum.so ;; slots) LP=tools/lib_passaslots/libhipquorum.so ;; *) LP=dragonboat_amd/lib/libhipquorum.so ;; esac
  ( export HQ_LIB_PATH=$PWD/$LP COMPACT=1 LEG=step5 W=$W STEPS=6; timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/$n -o run -- python3 tools/step_probe.py > gpurun_out/${n}.log 2>&1 ) || { tail gpurun_out/${n}.log; exit 4; }
  python3 tools/step_timeline.py gpurun_out/$n 6 $W > gpurun_out/${n}_timeline.txt 2>&1 || exit 5
  echo "== $L W=$W"; grep "step 5" gpurun_out/${n}.log; head -8 gpurun_out/${n}_timeline.txt
done
done
