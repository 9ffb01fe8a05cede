#!/bin/bash
# Round 5: the whole GPU suite on the two-rows-per-lane build.
set -o pipefail
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
