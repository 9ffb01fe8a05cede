#!/bin/bash
# Round 5 pre-final check: the whole GPU suite with test ids and the loaded in-tree
# libraries, smoke (with the affine path), one configs[2] bench line.
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
ANYSEQ_MAPS_OUT=$O/loaded_libs.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); import sys; sys.path.insert(0, 'tests'); import conftest; [print('loaded', r, d) for r, d in conftest.loaded_libraries()]" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-anchor --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
tail -2 $O/pytest.log; cat $O/loaded_libs.txt; tail -3 $O/smoke.log; grep -o '"value": [0-9.]*' $O/c2.json
