# r05f: PMC passes over the step5 device step, W = 1 (what bounds pass A)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export LEG=step5 W=1 STEPS=4
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r05f_counters.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT_LDS_ONLY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/r05f_p$i -o run -- python3 tools/step_probe.py > gpurun_out/r05f_p$i.log 2>&1 || { tail -5 gpurun_out/r05f_p$i.log; echo "pass $i failed"; }
done
echo done
