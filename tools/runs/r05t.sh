#!/bin/bash
# Round 5: the tail launches' phases (ANYSEQ_TAIL_STAMPS) on configs[2].
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
ANYSEQ_TAIL_STAMPS=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-anchor --steps 2 --warmup 1 > $O/c2.json 2> $O/c2.err || exit 1
tail -9 $O/c2.err
