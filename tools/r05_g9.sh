# r05i: engine tests, the engine's per-launch overhead (post + drain vs run), the default line
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05i_engine_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_engine_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/engine_overhead.py > gpurun_out/r05i_eng_over.log 2>&1 || exit 4
cat gpurun_out/r05i_eng_over.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --extra= --no-cpu --steps 20 --warmup 5 --detail-out gpurun_out/r05i_detail_$i.json > gpurun_out/r05i_bench_$i.log 2>&1 || exit 5
grep '^{"metric"' gpurun_out/r05i_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; f=d['fused_window']
print('value %.4g frac %.4f' % (d['value'], d['roofline']['frac']), 'engine us/step', e['window_kernel_us_per_step'], 'fused %.3f frac %.4f' % (f['median_kernel_us_per_step'], f['frac']), 'launch %.4f' % d['launch_per_step']['frac'], 'eq', e['engine_equals_launch_set0'])"
done
