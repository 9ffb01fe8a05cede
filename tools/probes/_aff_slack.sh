#!/bin/bash
# affine band-chain timeline at several slack settings (diagnostic, stamps build)
set -e
mkdir -p gpurun_out/$1
for sl in ${@:2}; do
  ANYSEQ_SLACK=$sl timeout -k 10 100 python3 tools/probes/_aff_timeline.py gpurun_out/$1/tl_s$sl local 65536 > gpurun_out/$1/tl_s$sl.log 2>&1
  echo "== slack $sl"; grep -E "launch|misses|steady duration|start lag:|end lag:" gpurun_out/$1/tl_s$sl.log | head -6
done
