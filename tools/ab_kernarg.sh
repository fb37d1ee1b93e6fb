# A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime's default, on
# the default headline (engine windows: the launch reads ~2 KB of descriptors from its arguments)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for V in 0 1; do
  ( export HIP_FORCE_DEV_KERNARG=$V; timeout -k 10 200 python3 -u bench.py --extra= --no-cpu --steps 20 --warmup 5 --detail-out gpurun_out/ab_kernarg_$V.json > gpurun_out/ab_kernarg_${V}_$i.log 2>&1 ) || exit 3
  grep '^{"metric"' gpurun_out/ab_kernarg_${V}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; f=d['fused_window']
print('DEV_KERNARG=$V', 'engine us/step', e['window_kernel_us_per_step'], 'frac %.4f' % e['frac'], 'fused %.3f frac %.4f' % (f['median_kernel_us_per_step'], f['frac']), 'launch %.4f' % d['launch_per_step']['frac'])"
done
done
