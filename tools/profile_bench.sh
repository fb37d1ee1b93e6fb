#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats of the bench command, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass). Each step has its own time limit;
# the script stops at the first failure. The trace runs the driver's command (--steps 20 --warmup 5
# unless STEPS / WARMUP say otherwise).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${1:-c2}
OUT=gpurun_out/prof_$W
# kernel legs (bench extras) ride along the headline workload
case $W in rim|rimt|rimtc|cq|cqp|c4pq|ing|ingo|ingu) ARGS="--workload c2tl --extra $W" ;; *) ARGS="--workload $W --extra=" ;; esac
mkdir -p $OUT
set -o pipefail
echo "== kernel trace ($W)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $ARGS --no-cpu --steps ${STEPS:-20} --warmup ${WARMUP:-5} --detail-out $OUT/trace_detail.json > $OUT/trace_stdout.log 2>&1 || exit $?
tail -n 1 $OUT/trace_stdout.log
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C ($W)"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- \
    python3 bench.py $ARGS --no-cpu --steps 40 --warmup 4 --detail-out $OUT/pmc_${C}_detail.json > $OUT/pmc_${C}_stdout.log 2>&1 || exit $?
done
find $OUT -name "*.csv" | sort
