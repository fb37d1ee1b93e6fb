# r05j: the default line twice (headline fused; engine windows post one step per call)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --extra= --no-cpu --steps 20 --warmup 5 --detail-out gpurun_out/r05j_detail_$i.json > gpurun_out/r05j_bench_$i.log 2>&1 || exit 5
grep '^{"metric"' gpurun_out/r05j_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; f=d['fused_window']
print('value %.4g frac %.4f mode %s' % (d['value'], d['roofline']['frac'], d['config']['headline_mode']), 'engine us/step', e['window_kernel_us_per_step'], 'frac %.4f' % e['frac'], 'fused %.3f frac %.4f' % (f['median_kernel_us_per_step'], f['frac']), 'launch %.4f' % d['launch_per_step']['frac'], 'eq', e['engine_equals_launch_set0'], 'sig', d['engine_signal']['median_ms_per_step'])"
done
