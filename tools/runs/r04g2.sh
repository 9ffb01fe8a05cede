#!/bin/bash
# Round 4: hipGraph replay of the device-planned levels (ANYSEQ_GRAPH=1): parity, then A/B
# against the plain enqueue, interleaved.
set -o pipefail
O=gpurun_out/r04g2; mkdir -p $O
ANYSEQ_GRAPH=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for g in 0 1; do
    ANYSEQ_GRAPH=$g timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_g${g}_r$rep.json 2> $O/c2_g${g}_r$rep.err || exit 1
  done
done
