#!/bin/bash
# Round 6: rocprofv3 evidence of the final tree: the headline (c3mtl, the driver's command) trace +
# FETCH_SIZE / WRITE_SIZE passes, and the same for the engine windows. Summaries by
# tools/summarize_profiles.py r06f c3mtl c3mtl-engine.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/profile_bench.sh c3mtl > gpurun_out/profile_c3mtl.log 2>&1 || exit $?
bash tools/profile_engine.sh c3mtl > gpurun_out/profile_c3mtl-engine.log 2>&1 || exit $?
echo all ok
