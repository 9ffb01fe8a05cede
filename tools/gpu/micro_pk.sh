#!/bin/bash
# the packed 16-bit step projection against the product's three-row loop (tools/micro/mix_micro.hip)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
MIX_ONLY_PK=1 timeout -k 10 180 tools/micro/bin/mix_g > $O/mix_g.txt 2>&1 || { tail -20 $O/mix_g.txt; exit 1; }
cat $O/mix_g.txt
