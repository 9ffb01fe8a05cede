#!/bin/bash
# Round 5: is the I/O wave's subject work what slows the HBM hop?  Diagnostic
# ANYSEQ_IO_SKEW=-1 (no subject staging / skewed copy: wrong scores, timing only) against
# the default, affine local score; band timelines of both (stamps build, with the band-end
# events: producer's last half published -> consumer sees it).
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-anchor --config 1 --kind local --gap-open -2 --steps 10 --warmup 3"
for rep in 1 2; do
  timeout -k 10 120 $B > $O/afl_def_r$rep.json 2> $O/afl_def_r$rep.err || exit 1
  ANYSEQ_IO_SKEW=-1 timeout -k 10 120 $B > $O/afl_noskew_r$rep.json 2> $O/afl_noskew_r$rep.err || exit 1
done
timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl_def > $O/timeline_def.txt 2>&1 || exit 1
ANYSEQ_IO_SKEW=-1 timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl_noskew > $O/timeline_noskew.txt 2>&1 || exit 1
