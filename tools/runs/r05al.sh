#!/bin/bash
# Round 5: linear global / local scores through the affine fill by default -- the whole GPU suite, configs[1] / [2].
set -o pipefail
O=gpurun_out/r05al; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-anchor > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
for f in c1 c2; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);c=d['config'];print('$f', d['value'], d['ms_per_step'], c.get('score'), d['roofline'].get('frac'), d['roofline'].get('kernel'))"; done
