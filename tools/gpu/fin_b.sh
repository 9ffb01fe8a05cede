#!/bin/bash
# Round-end evidence, part B: the profile set (bench lines, kernel traces, PMC passes).
set -o pipefail
mkdir -p gpurun_out/prof_$1
timeout -k 10 1100 bash tools/profile.sh $1 > gpurun_out/prof_$1/profile.log 2>&1 || { tail -20 gpurun_out/prof_$1/profile.log; exit 1; }
tail -3 gpurun_out/prof_$1/profile.log
