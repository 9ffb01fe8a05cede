#!/bin/bash
# Round 5: the two-rows-per-lane projection of the affine loop (mix_micro R2 variants).
set -o pipefail
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 120 tools/micro/bin/mix_micro_lds > $O/mix_lds.txt 2>&1 || exit 1
grep "WGs 256" $O/mix_lds.txt | grep "FULL\|VALU \|R2"
