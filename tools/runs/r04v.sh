#!/bin/bash
# Round 4: which half of the new band ends breaks the local construct -- the fused end
# (ANYSEQ_AFFINE_ASM=65: new end, round-3 start) or the spin-free start (=33)?
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
for a in 97 65 33 1; do
  ANYSEQ_AFFINE_ASM=$a timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_affine_construct.py -k "random or multi_group or transposed" > $O/pytest_a$a.log 2>&1
  echo "affasm $a: $(tail -1 $O/pytest_a$a.log)"
done
