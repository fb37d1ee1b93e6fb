#!/bin/bash
# rocprofv3 evidence for the default bench line (headline mode "engine"): the driver's command
# (--steps 20 --warmup 5) under --kernel-trace --stats, then one PMC pass per counter group
# (FETCH_SIZE, WRITE_SIZE) of the same command. tools/summarize_profiles.py ROUND c3mtl-engine
# turns the engine's window launches into per-step figures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${1:-c3mtl}
OUT=gpurun_out/prof_${W}-engine
ARGS="--workload $W --extra= --steps 20 --warmup 5 --no-cpu"
mkdir -p $OUT
set -o pipefail
echo "== kernel trace ($W, engine)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $ARGS --detail-out $OUT/trace_detail.json > $OUT/trace_stdout.log 2>&1 || exit $?
tail -n 1 $OUT/trace_stdout.log | cut -c1-300
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C ($W, engine)"
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- \
    python3 bench.py $ARGS --detail-out $OUT/pmc_${C}_detail.json > $OUT/pmc_${C}_stdout.log 2>&1 || exit $?
done
find $OUT -name "*.csv" | sort
