#!/bin/bash
# rocprofv3 evidence only (no tests / bench): PROF="c3 ..." bash tools/prof_only.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for W in ${PROF:-c2}; do bash tools/profile_bench.sh $W > gpurun_out/profile_$W.log 2>&1 || { tail gpurun_out/profile_$W.log; exit 4; }; done
echo prof-done
