#!/bin/bash
# Round 4: the capture-free band end now also for bands with a best of every cell (blocks
# past the last chunk read a "minus infinity" top row): parity under ANYSEQ_AFFINE_ASM=65
# (fused end, round-3 start), then A/B 97 / 65 / 1 interleaved.
set -o pipefail
O=gpurun_out/r04f2; mkdir -p $O
ANYSEQ_AFFINE_ASM=65 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for a in 97 65 1; do
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_a${a}_r$rep.json 2> $O/c2_a${a}_r$rep.err || exit 1
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_a${a}_r$rep.json 2> $O/afl_a${a}_r$rep.err || exit 1
  done
done
