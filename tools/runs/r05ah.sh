#!/bin/bash
# Round 5: rows per lane chosen among 1-3 (auto): the multi-row tests, configs[4] / [3] / [2].
set -o pipefail
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine_r2.py tests/test_gpu_affine.py > $O/r23.log 2>&1 || { tail -30 $O/r23.log; exit 1; }
tail -2 $O/r23.log
timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-anchor > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
for f in c4 c3 c2; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);c=d['config'];print('$f', d['value'], d['ms_per_step'], c.get('score'), c.get('fill_multi_row_launches_per_step'), c.get('fill_rows_per_lane_max'), c.get('fill_launches_per_step'))"; done
