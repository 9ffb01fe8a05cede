#!/bin/bash
# GPU box: A/B of the affine I/O wave's idle sleep (anyseq_amd/libanyseq_sleep{2,4}.so, built
# with -DANYSEQ_IO_SLEEP=2 / 4) against the product build: affine construct tests, then
# configs[2] and affine local score lines, alternating.  Usage: bash tools/gpu_r03j.sh
set -e
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
for L in sleep2 sleep4; do
  ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_$L.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$L.log 2>&1
  tail -1 $OUT/pytest_$L.log
done
for i in 1 2; do
  for L in libanyseq libanyseq_sleep2 libanyseq_sleep4; do
    ANYSEQ_LIB=$PWD/anyseq_amd/$L.so timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-anchor > $OUT/c2_${L}_$i.json 2> $OUT/c2_${L}_$i.err
    ANYSEQ_LIB=$PWD/anyseq_amd/$L.so timeout -k 10 120 python3 -u bench.py --config 1 --kind local --gap-open -2 --no-cpu-baseline > $OUT/al_${L}_$i.json 2> $OUT/al_${L}_$i.err
  done
done
echo done
