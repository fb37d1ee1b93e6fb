#!/bin/bash
# A/B of the binned table ingest (hq_table.hip k_bin / k_apply): for the default build and each
# variant in $VARIANTS — a library tools/lib_<v>/libhipquorum.so (the Makefile's binab / bintpb
# targets) or an environment setting NAME=VALUE (e.g. HQ_BIN_GRID=512) — one rocprofv3 kernel
# trace of the ing leg; prints each kernel's average duration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LEG=${LEG:-ing}
VARIANTS=${VARIANTS:-binab1 binab2 binab3 bintpb5 bintpb4}
OUT=gpurun_out/ab_bin
mkdir -p $OUT
for v in default $VARIANTS; do
  unset HQ_LIB_PATH HQ_BIN_GRID HQ_BIN_TPB
  case $v in
    default) ;;
    *=*) export "$v" ;;
    *) export HQ_LIB_PATH=tools/lib_$v/libhipquorum.so ;;
  esac
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- \
    python3 bench.py --workload c2tl --extra $LEG --no-cpu --steps 40 --warmup 5 \
    --detail-out $OUT/$v/detail.json > $OUT/$v.log 2>&1 || exit $?
  echo "== $v"
  grep -h "k_bin\|k_apply\|k_table_ingest" $OUT/$v/run_kernel_stats.csv | \
    python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print('  %-40s avg %8.2f us' % (r['Name'].split('(')[1].split(')')[0].split('::')[-1]
                                    if r['Name'].startswith('void') else r['Name'][:40],
                                    float(r['AverageNs']) / 1e3))
" $OUT/$v/run_kernel_stats.csv | grep -v "k_synth\|k_tile\|fill\|k_commit"
done
