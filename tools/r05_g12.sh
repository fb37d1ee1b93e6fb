# r05m: device step / engine / encoder tests, then the default line with the step legs
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05m}
timeout -k 10 500 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_step_leg.py tests/test_gpu_engine.py tests/test_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --extra step,step5 --detail-out gpurun_out/${T}_detail.json > gpurun_out/${T}_bench.log 2>&1 || exit 5
grep '^{"metric"' gpurun_out/${T}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; f=d['fused_window']
print('value %.4g frac %.4f mode %s' % (d['value'], d['roofline']['frac'], d['config']['headline_mode']), 'engine us/step', e['window_kernel_us_per_step'], 'frac %.4f' % e['frac'], 'launch %.4f' % d['launch_per_step']['frac'])
for k, v in d['extra'].items(): print(k, json.dumps(v)[:600])"
