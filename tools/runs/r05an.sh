#!/bin/bash
# Round 5: zero-open left border forced at column -1 (semiglobal virtual prologue): the GPU suite, semiglobal timing.
set -o pipefail
O=gpurun_out/r05an; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0; do
ANYSEQ_FORCE_LB=$v timeout -k 10 200 python -u bench.py --config 1 --kind semiglobal --gap-open -2 --steps 5 --warmup 2 --no-cpu-baseline > $O/as_$v.json 2> $O/as_$v.err || { tail -20 $O/as_$v.err; exit 1; }
ANYSEQ_FORCE_LB=$v ANYSEQ_LIN_AFF=2 timeout -k 10 200 python -u bench.py --config 1 --kind semiglobal --steps 5 --warmup 2 --no-cpu-baseline > $O/ls_$v.json 2> $O/ls_$v.err || { tail -20 $O/ls_$v.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --config 1 --kind semiglobal --steps 5 --warmup 2 --no-cpu-baseline > $O/ls_lin.json 2> $O/ls_lin.err || { tail -20 $O/ls_lin.err; exit 1; }
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['config'].get('score'))"; done
