#!/bin/bash
# configs[2]: two / three rows per lane at four compute waves (the score launch is chain-bound: fewer, taller bands);
# the affine local score launch alone (config 1 --kind local --gap-open -2) the same way.
set -o pipefail
O=gpurun_out/r05ap; mkdir -p $O
run() { local tag=$1 args=$2; shift 2; env "$@" timeout -k 10 120 python -u bench.py $args --steps 5 --warmup 2 --no-cpu-baseline --no-anchor > $O/$tag.json 2> $O/$tag.err || exit 1; echo "$tag $(python -c "import json,sys; d=json.load(open('$O/$tag.json')); print(d['value'], d['ms_per_step'], d['config'].get('fill_gcups'), d['config'].get('fill_rows_per_lane_max'), d['config'].get('fill_multi_row_launches_per_step'))")"; }
C1="--config 1 --kind local --gap-open -2"
run base "" X=1
run nwa4r2 "" ANYSEQ_NWA=4 ANYSEQ_AFF_ROWS=2
run nwa4r3 "" ANYSEQ_NWA=4 ANYSEQ_AFF_ROWS=3
run s_base "$C1" X=1
run s_nwa4 "$C1" ANYSEQ_NWA=4
run s_nwa4r2 "$C1" ANYSEQ_NWA=4 ANYSEQ_AFF_ROWS=2
run s_nwa4r3 "$C1" ANYSEQ_NWA=4 ANYSEQ_AFF_ROWS=3
run s_nwa7r2 "$C1" ANYSEQ_NWA=7 ANYSEQ_AFF_ROWS=2
