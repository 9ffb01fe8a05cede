#!/bin/bash
# Round 5: linear scores through the affine fill (linear loop / affine loop): parity, then configs[1] timing.
set -o pipefail
O=gpurun_out/r05ak; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear_affine.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python -u bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
ANYSEQ_LIN_AFF=1 timeout -k 10 200 python -u bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/c1_la.json 2> $O/c1_la.err || { tail -20 $O/c1_la.err; exit 1; }
ANYSEQ_LIN_AFF=1 ANYSEQ_LIN_LOOP=0 timeout -k 10 200 python -u bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/c1_aa.json 2> $O/c1_aa.err || { tail -20 $O/c1_aa.err; exit 1; }
for k in local semiglobal; do
timeout -k 10 200 python -u bench.py --config 1 --kind $k --steps 5 --warmup 2 --no-cpu-baseline > $O/c1_$k.json 2> $O/c1_$k.err || { tail -20 $O/c1_$k.err; exit 1; }
ANYSEQ_LIN_AFF=1 timeout -k 10 200 python -u bench.py --config 1 --kind $k --steps 5 --warmup 2 --no-cpu-baseline > $O/c1_la_$k.json 2> $O/c1_la_$k.err || { tail -20 $O/c1_la_$k.err; exit 1; }
done
for f in c1 c1_la c1_aa c1_local c1_la_local c1_semiglobal c1_la_semiglobal; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);c=d['config'];print('$f', d['value'], d['ms_per_step'], c.get('score'))"; done
