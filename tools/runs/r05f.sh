#!/bin/bash
# Round 5: (1) LEAN=2 (subject-prefetch wait every other block) parity and A/B against
# LEAN=1; (2) the I/O wave's hand-off knobs on the new loop (priority 3 for its hand-off
# step, skewed blocks per pass while a poll is out, staging mode), affine local score.
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
EXP=$PWD/anyseq_amd/libanyseq_exp.so
ANYSEQ_LIB=$EXP timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest_exp.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
for rep in 1 2; do
  for lib in libanyseq.so libanyseq_exp.so; do
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_${lib%.so}_r$rep.json 2> $O/c2_${lib%.so}_r$rep.err || exit 1
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_${lib%.so}_r$rep.json 2> $O/afl_${lib%.so}_r$rep.err || exit 1
  done
  for kv in PRIO=3 IO_SKEW=1 IO_SKEW=2 IO_SKEW=4 IO_STAGE=2 PRIO=0; do
    env ANYSEQ_$kv timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_${kv}_r$rep.json 2> $O/afl_${kv}_r$rep.err || exit 1
  done
done
