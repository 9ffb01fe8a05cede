#!/bin/bash
# per-step ds_write publish vs the DPP shift register (tools/micro/mix_micro.hip, DSFULL)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
MIX_ONLY_DS=1 timeout -k 10 120 tools/micro/bin/mix_l > $O/mix_l.txt 2>&1 || { tail -20 $O/mix_l.txt; exit 1; }
cat $O/mix_l.txt
