# A/B: the producer's encode threads (BENCH_HQ_ENCODE_THREADS) on the step legs, two rounds
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for V in 14 15 16; do
  ( export BENCH_HQ_ENCODE_THREADS=$V; timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --extra step,step5 --no-cpu --detail-out gpurun_out/ab_enct_${V}_$i.json > gpurun_out/ab_enct_${V}_$i.log 2>&1 ) || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_enct_${V}_$i.json'))
for rec in d['extra']:
    if 'latency_ms' not in rec: continue
    L=rec['latency_ms']; ph=rec['e2e_phases']
    print('T=$V', rec['name'], 'e2e p50', {k: L[k]['p50'] for k in L if k.startswith('e2e')}, 'enc', {w: ph[w]['median'].get('encode_max_ms') for w in ph}, 'thr', {w: ph[w]['median'].get('throttled_ms_total') for w in ph})"
done
done
