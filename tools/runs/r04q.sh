#!/bin/bash
# Round 4: band timeline on the current defaults (issue priority 1, staging 3); A/B of the
# start slack (ANYSEQ_SLACK 0/1/2) interleaved on one box; configs[4] at N=1.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for sl in 0 1 2; do
    ANYSEQ_SLACK=$sl timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_s${sl}_r$rep.json 2> $O/c2_s${sl}_r$rep.err || exit 1
    ANYSEQ_SLACK=$sl timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_s${sl}_r$rep.json 2> $O/afl_s${sl}_r$rep.err || exit 1
  done
done
timeout -k 10 300 $B --config 4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 1
