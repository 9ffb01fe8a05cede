#!/bin/bash
# Round 5: configs[4] / [3] N=1 with two rows per lane (auto) against one row (ANYSEQ_AFF_ROWS=1), one box.
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_r2.json 2> $O/c4_r2.err || { tail -20 $O/c4_r2.err; exit 1; }
echo "c4 R2"; python3 -c "import json;d=json.loads(open('$O/c4_r2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
ANYSEQ_AFF_ROWS=1 timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_r1.json 2> $O/c4_r1.err || { tail -20 $O/c4_r1.err; exit 1; }
echo "c4 R1"; python3 -c "import json;d=json.loads(open('$O/c4_r1.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3_r2.json 2> $O/c3_r2.err || { tail -20 $O/c3_r2.err; exit 1; }
echo "c3 R2"; python3 -c "import json;d=json.loads(open('$O/c3_r2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
echo "c2"; python3 -c "import json;d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
