#!/bin/bash
# round 6: GPU suite on the current build, A/B against HEAD's library, a configs[2] kernel trace
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash tools/gpu/ab2.sh $1 head,prod "" || exit 1
bash tools/gpu/trace_c2.sh $1
