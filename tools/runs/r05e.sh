#!/bin/bash
# Round 5: band timeline of the lean loop with the fused end (stamps build), 65536^2 local
# affine score; kernel-trace of configs[2] on the new defaults.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-anchor > $O/trace_bench.json 2> $O/trace.err || exit 1
