#!/bin/bash
# Round 5 milestone (code rows + lean loop + fused end): the whole GPU suite with test ids,
# smoke, the profile set (bench lines, kernel traces, PMC passes), configs[3] / [4] N=1.
set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1500 bash tools/profile.sh r05j > $O/profile.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
