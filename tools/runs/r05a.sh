#!/bin/bash
# Round 5 start: the inherited tree on a fresh box (GPU suite with test ids, smoke, default bench).
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
