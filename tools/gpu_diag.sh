#!/bin/bash
# One diagnostic pass on the GPU box: the GPU suite under a kernel trace, HIP
# runtime errors to stderr, failure context from the engine (fill_summary).
# Usage (repo root, on the box): bash tools/gpu_diag.sh <tag> [pytest args...]
set -o pipefail
TAG=${1:-diag}
shift
OUT=gpurun_out/diag_$TAG
mkdir -p $OUT
export TMPDIR=/tmp AMD_LOG_LEVEL=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
    python3 -u -m pytest ${@:-tests -m gpu} -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
exit $rc
