#!/bin/bash
# Round 5: which VALU mixes co-issue from two waves of one SIMD (item 4).
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 120 tools/micro/bin/coissue_micro > $O/coissue.txt 2>&1 || exit 1
cat $O/coissue.txt
