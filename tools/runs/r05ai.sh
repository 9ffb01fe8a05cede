#!/bin/bash
# Round 5: eight compute waves without the I/O wave (self-forwarding first bands): parity, then configs[4] / [3].
set -o pipefail
O=gpurun_out/r05ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine_r2.py tests/test_gpu_affine.py tests/test_gpu_shard_affine.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
ANYSEQ_SELF_FWD=1 timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_sf.json 2> $O/c4_sf.err || { tail -20 $O/c4_sf.err; exit 1; }
timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
ANYSEQ_SELF_FWD=1 timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_sf.json 2> $O/c3_sf.err || { tail -20 $O/c3_sf.err; exit 1; }
for f in c4_sf c4 c3_sf; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);c=d['config'];print('$f', d['value'], d['ms_per_step'], c.get('score'), c.get('fill_rows_per_lane_max'))"; done
