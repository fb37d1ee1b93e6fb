#!/bin/bash
# One GPU-box session: parity tests, smoke, bench. Stops at the first fault/timeout/abort;
# plain test failures (pytest exit 1) still let the bench run so both results come back.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
rc=$?; if fatal $rc; then exit $rc; fi
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
rc=$?; if fatal $rc; then exit $rc; fi
step bench 400 python -u bench.py
rc=$?; if fatal $rc; then exit $rc; fi
cat gpurun_out/bench.log | tail -n 1
