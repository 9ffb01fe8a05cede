#!/bin/bash
# Round 5: the fused band end opened to every-cell bests (I/O-wave pad past the last
# granule + masked top row past the last chunk): parity under affine_asm 1 / 65, the
# round-4 race probe, then A/B 97 / 65 / 1 interleaved on one box.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest.log 2>&1 || exit 1
for a in 1 65; do
  ANYSEQ_AFFINE_ASM=$a timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_golden.py > $O/pytest_a$a.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/probes/_fused_best_race.py > $O/race.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for a in 97 65 1; do
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_a${a}_r$rep.json 2> $O/c2_a${a}_r$rep.err || exit 1
    ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_a${a}_r$rep.json 2> $O/afl_a${a}_r$rep.err || exit 1
  done
done
