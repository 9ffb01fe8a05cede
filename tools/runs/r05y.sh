#!/bin/bash
# Round 5: the whole GPU suite with the fill events off (ANYSEQ_FILL_EVENTS=0: the bench's
# timed path) -- every engine path synchronises on its copy events instead.
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
ANYSEQ_FILL_EVENTS=0 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
tail -2 $O/pytest.log
