#!/bin/bash
# Round 4: capture-free asm epilogue (bands whose last-column state nobody reads): parity,
# A/B against the capturing epilogue (ANYSEQ_AFFINE_ASM 1 vs 33) interleaved, timeline.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_shard_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for a in 1 33; do
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_a${a}_r$rep.json 2> $O/c2_a${a}_r$rep.err || exit 1
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_a${a}_r$rep.json 2> $O/afl_a${a}_r$rep.err || exit 1
  done
done
ANYSEQ_AFFINE_ASM=1 timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
