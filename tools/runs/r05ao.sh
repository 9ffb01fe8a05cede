#!/bin/bash
# configs[2] A/B over the affine fill's shape knobs (rows per lane, compute waves, self-forwarding).
set -o pipefail
O=gpurun_out/r05ao; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-anchor > $O/$tag.json 2> $O/$tag.err || exit 1; echo "$tag $(python -c "import json,sys; d=json.load(open('$O/$tag.json')); print(d['value'], d['ms_per_step'], d['config'].get('fill_gcups'), d['config'].get('fill_rows_per_lane_max'), d['roofline'].get('frac'))")"; }
run base X=1
run sf0 ANYSEQ_SELF_FWD=0
run r2 ANYSEQ_AFF_ROWS=2
run r3 ANYSEQ_AFF_ROWS=3
run r1 ANYSEQ_AFF_ROWS=1
run nwa4 ANYSEQ_NWA=4
run nwa7 ANYSEQ_NWA=7
run nwa8 ANYSEQ_NWA=8
run nwa8r2 ANYSEQ_NWA=8 ANYSEQ_AFF_ROWS=2
run nwa7r2 ANYSEQ_NWA=7 ANYSEQ_AFF_ROWS=2
