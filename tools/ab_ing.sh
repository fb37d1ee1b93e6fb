cd $GRAFT_REPO_ROOT
run() { timeout -k 10 120 python3 -c "
import bench
d=bench.Dist(); r=bench.run_kernel_leg('ing', 50, 5, d, parity_threads=0)
print('%.2f us/step' % (r['ms_per_step']*1e3 if 'ms_per_step' in r else -1), 'frac %.4f' % r['roofline_frac'], 'value %.3e' % r['value'])" 2>&1 | tail -1; }
for r in 1 2 3; do
  echo -n "round $r default: "; run || exit 1
  echo -n "round $r T512 tpb5 grid512: "; HQ_BIN_APPLY_T=512 HQ_BIN_TPB=5 HQ_BIN_GRID=512 run || exit 1
  echo -n "round $r T512 tpb5 grid256: "; HQ_BIN_APPLY_T=512 HQ_BIN_TPB=5 HQ_BIN_GRID=256 run || exit 1
  echo -n "round $r T1024 tpb5 grid256: "; HQ_BIN_TPB=5 run || exit 1
done
HQ_BIN_APPLY_T=512 HQ_BIN_TPB=5 HQ_BIN_GRID=512 timeout -k 10 400 python3 -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_table.py tests/test_gpu_ingest.py 2>&1 | tail -2
