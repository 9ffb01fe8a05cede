#!/bin/bash
# Round 4: A/B of the affine I/O wave's issue priority (ANYSEQ_PRIO 0/1/3) and skew blocks per
# polling pass (ANYSEQ_IO_SKEW 8/2/32), interleaved on one box; SIMD placement probe.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 120 tools/micro/bin/aff_loop_micro > $O/aff_loop_micro.txt 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for cfg in "0 8" "1 8" "3 8" "0 2" "0 32"; do
    set -- $cfg
    ANYSEQ_PRIO=$1 ANYSEQ_IO_SKEW=$2 timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_p$1_s$2_r$rep.json 2> $O/c2_p$1_s$2_r$rep.err || exit 1
    ANYSEQ_PRIO=$1 ANYSEQ_IO_SKEW=$2 timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_p$1_s$2_r$rep.json 2> $O/afl_p$1_s$2_r$rep.err || exit 1
  done
done
