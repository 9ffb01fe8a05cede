#!/bin/bash
# configs[2] kernel trace (per-launch durations of the construct's levels)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-anchor > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
ls -R $O | head
