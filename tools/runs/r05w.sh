#!/bin/bash
# Round 5: launch gaps around a large kernel (tools/micro/gap_micro.hip) under the kernel trace.
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- tools/micro/bin/gap_micro > $O/gap.log 2>&1 || exit 1
python3 tools/micro/gap_report.py $O/trace/run_kernel_trace.csv | tee $O/gap_report.txt
