#!/bin/bash
# Round 6: debug of the consecutive-run differential: the product library and a build without
# take_run, on the failing seed / feed. Outputs gpurun_out/r06o/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
SEED=31 FEED=stream timeout -k 10 200 python -u tools/dbg_runs.py > $O/dbg_take.log 2>&1 || exit $?
HQ_LIB_PATH=tools/lib_notakerun/libhipquorum.so SEED=31 FEED=stream timeout -k 10 200 python -u tools/dbg_runs.py > $O/dbg_notake.log 2>&1 || exit $?
cat $O/dbg_take.log $O/dbg_notake.log
