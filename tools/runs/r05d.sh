#!/bin/bash
# Round 5: (1) parity of the default build with the fused end opened to every-cell bests
# and the positive-mismatch fixes, under the default ends and the fused ones; (2) the
# lean affine loop (ANYSEQ_GEN_LEAN, libanyseq_lean.so): its parity and its isolated
# cycles per step beside the default loop's; (3) A/B on one box, interleaved: library
# {default, lean} x band end {97 round-3 ends, 1 fused end + spin-free start}.
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
AFF="tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py"
$T -rA $AFF > $O/pytest.log 2>&1 || exit 1
ANYSEQ_AFFINE_ASM=1 $T $AFF tests/test_gpu_golden.py > $O/pytest_a1.log 2>&1 || exit 1
ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_lean.so $T $AFF > $O/pytest_lean.log 2>&1 || exit 1
ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_lean.so ANYSEQ_AFFINE_ASM=1 $T $AFF > $O/pytest_lean_a1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probes/_fused_best_race.py > $O/race.log 2>&1 || exit 1
timeout -k 10 120 tools/micro/bin/aff_loop_micro > $O/loop_default.txt 2>&1 || exit 1
timeout -k 10 120 tools/micro/bin/aff_loop_micro_lean > $O/loop_lean.txt 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for lib in libanyseq.so libanyseq_lean.so; do
    for a in 97 1; do
      tag=${lib%.so}_a$a
      ANYSEQ_LIB=$PWD/anyseq_amd/$lib ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_${tag}_r$rep.json 2> $O/c2_${tag}_r$rep.err || exit 1
      ANYSEQ_LIB=$PWD/anyseq_amd/$lib ANYSEQ_AFFINE_ASM=$a timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_${tag}_r$rep.json 2> $O/afl_${tag}_r$rep.err || exit 1
    done
  done
done
