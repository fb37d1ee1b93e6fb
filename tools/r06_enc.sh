#!/bin/bash
# Round 6: the producer's encode tail — the step5 worker's step beside the encode
# (tools/late_probe.py conc) on the encode-profiling build (tools/lib_encprof/, -DHQ_ENC_PROF),
# the encoder's chunks per thread alternated step by step (AB: HQ_ENC_CHUNKS values; 1 = one
# range per thread, round 5's static split). Outputs under gpurun_out/r06w/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06w
mkdir -p $O
AB=8,1 MODES=conc STEPS=300 ROWS=1 HQ_LIB_PATH=tools/lib_encprof/libhipquorum.so timeout -k 10 150 python3 -u tools/late_probe.py > $O/enc_ab81.log 2> $O/enc_ab81.err || exit $?
AB=8,4,2,1 MODES=conc STEPS=400 ROWS=1 HQ_LIB_PATH=tools/lib_encprof/libhipquorum.so timeout -k 10 150 python3 -u tools/late_probe.py > $O/enc_ab8421.log 2> $O/enc_ab8421.err || exit $?
echo all ok
