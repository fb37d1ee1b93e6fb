# A/B by kernel trace: pass A's duration (k_step_jobs<false, ...>) with the tree's library and
# with tools/lib_ab/libhipquorum_base.so, step5 W=1 (one job), two alternated rounds
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for L in base new; do
  d=gpurun_out/abpa_${L}_$i
  ( if [ $L = base ]; then export HQ_LIB_PATH=$PWD/tools/lib_ab/libhipquorum_base.so; fi
    export LEG=${LEG:-step5} W=1 STEPS=10
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/step_probe.py > $d.log 2>&1 ) || { tail -3 $d.log; exit 3; }
  python3 -c "
import csv,statistics
rows=list(csv.DictReader(open('$d/run_kernel_trace.csv')))
for k in ('k_step_jobs<false', 'k_step_lite_jobs', 'k_size_sums', 'k_step_jobs<true'):
    t=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if k in r['Kernel_Name']][3:]
    print('$L', k, 'median %.1f us (n=%d)' % (statistics.median(t), len(t)))"
done
done
