#!/bin/bash
# Round-end evidence, part A (the committed build, one fresh box): the whole GPU suite with
# test ids and the in-tree libraries it loaded, smoke, configs[3] and configs[4] bench lines.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
ANYSEQ_MAPS_OUT=$O/loaded_libs.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); import sys; sys.path.insert(0, 'tests'); import conftest; [print('loaded', r, d) for r, d in conftest.loaded_libraries()]" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
tail -2 $O/pytest.log; cat $O/loaded_libs.txt; tail -3 $O/smoke.log
