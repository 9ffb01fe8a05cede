#!/bin/bash
# affine band-chain timeline at several issue-priority settings (diagnostic, stamps build)
set -e
mkdir -p gpurun_out/$1
for pr in ${@:2}; do
  ANYSEQ_PRIO=$pr timeout -k 10 100 python3 tools/probes/_aff_timeline.py gpurun_out/$1/tl_p$pr local 65536 > gpurun_out/$1/tl_p$pr.log 2>&1
  echo "== prio $pr"; grep -E "launch|steady duration|start lag:|end lag:|hops" gpurun_out/$1/tl_p$pr.log | head -8
done
