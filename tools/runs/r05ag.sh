#!/bin/bash
# Round 5: configs[3] with three rows per lane (forced) against two (auto), and the GPU suite on this build.
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O
ANYSEQ_AFF_ROWS=3 timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_r3.json 2> $O/c3_r3.err || { tail -20 $O/c3_r3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_r2.json 2> $O/c3_r2.err || { tail -20 $O/c3_r2.err; exit 1; }
for f in c3_r3 c3_r2; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);c=d['config'];print('$f', d['value'], d['ms_per_step'], c.get('score'), c.get('fill_gcups'), c.get('fill_two_row_launches_per_step'), c.get('fill_launches_per_step'))"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
