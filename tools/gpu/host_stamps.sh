#!/bin/bash
# host-side phases of the configs[2] construct call (ANYSEQ_HOST_STAMPS)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
ANYSEQ_HOST_STAMPS=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-anchor --kernel-steps 1 > $O/bench.json 2> $O/stamps.txt || { tail -20 $O/stamps.txt; exit 1; }
grep "host stamps" $O/stamps.txt | tail -8
