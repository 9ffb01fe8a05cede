#!/bin/bash
# Round 4: band timelines at 65536 columns with 8192 / 65536 rows (64 / 512 bands per
# front) -- is the per-band slowdown along the chain a chain effect or a load effect? --
# and A/B of band 0's pace (ANYSEQ_THROTTLE 0/1/2 s_sleep-1 units per block), interleaved.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
for r in 8192 65536; do
  timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl_$r local $r > $O/timeline_$r.txt 2>&1 || exit 1
done
ANYSEQ_THROTTLE=1 timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl_thr1 local 65536 > $O/timeline_thr1.txt 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for t in 0 1 2; do
    ANYSEQ_THROTTLE=$t timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_t${t}_r$rep.json 2> $O/c2_t${t}_r$rep.err || exit 1
    ANYSEQ_THROTTLE=$t timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_t${t}_r$rep.json 2> $O/afl_t${t}_r$rep.err || exit 1
  done
done
