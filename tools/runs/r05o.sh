#!/bin/bash
# Round 5: the affine loop by instruction subset at one and two waves per SIMD (item 4).
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 120 tools/micro/bin/mix_micro_none > $O/mix_none.txt 2>&1 || exit 1
timeout -k 10 120 tools/micro/bin/mix_micro_lds > $O/mix_lds.txt 2>&1 || exit 1
cat $O/mix_none.txt $O/mix_lds.txt
