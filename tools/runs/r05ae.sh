#!/bin/bash
# Round 5: the three-rows-per-lane projection of the affine loop (mix_micro R3 variants).
set -o pipefail
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 150 tools/micro/bin/mix_micro_lds > $O/mix_lds.txt 2>&1 || exit 1
grep "WGs 256" $O/mix_lds.txt | grep "FULL\|VALU \|R2\|R3"
