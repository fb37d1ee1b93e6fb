# A/B: the jobs path's waiting thread polls (HQ_STEP_JOBS_SPIN_US=5000, default) or sleeps after 50 us
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for V in 50 5000; do
  ( export HQ_STEP_JOBS_SPIN_US=$V; timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-cpu --detail-out gpurun_out/ab_spin_${V}_$i.json > gpurun_out/ab_spin_${V}_$i.log 2>&1 ) || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_spin_${V}_$i.json'))
for rec in d['extra']:
    if 'latency_ms' not in rec: continue
    L=rec['latency_ms']; ph=rec['e2e_phases']
    print('spin=$V', rec['name'], 'dev p50', {k: L[k]['p50'] for k in L if k.startswith('dev')}, 'e2e p50', {k: L[k]['p50'] for k in L if k.startswith('e2e')}, 'thr', {w: ph[w]['median'].get('throttled_ms_total') for w in ph})"
done
done
