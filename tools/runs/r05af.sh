#!/bin/bash
# Round 5: three rows per lane -- projection (mix_micro R3), parity (forced), configs[4] / [2] timing.
set -o pipefail
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 150 tools/micro/bin/mix_micro_lds > $O/mix_lds.txt 2>&1 || exit 1
grep "WGs 256" $O/mix_lds.txt | grep "FULL\|VALU \|R2\|R3"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine_r2.py > $O/r23.log 2>&1 || { tail -30 $O/r23.log; exit 1; }
tail -2 $O/r23.log
ANYSEQ_AFF_ROWS=3 timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_r3.json 2> $O/c4_r3.err || { tail -20 $O/c4_r3.err; exit 1; }
timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_r2.json 2> $O/c4_r2.err || { tail -20 $O/c4_r2.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-anchor > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
for f in c4_r3 c4_r2 c2; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['config'].get('score'))"; done
