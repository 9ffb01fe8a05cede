#!/bin/bash
# GPU box: an experimental build (anyseq_amd/libanyseq_poll.so: pipelined hand-off polls)
# through the GPU suite, then configs[2] / affine local score lines of it and of the
# product build, alternating.  Usage: bash tools/gpu_r03i.sh
set -e
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
X=$PWD/anyseq_amd/libanyseq_poll.so
ANYSEQ_LIB=$X timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
for i in 1 2; do
  for L in $X $PWD/anyseq_amd/libanyseq.so; do
    t=$(basename $L .so)
    ANYSEQ_LIB=$L timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-anchor > $OUT/c2_${t}_$i.json 2> $OUT/c2_${t}_$i.err
    ANYSEQ_LIB=$L timeout -k 10 120 python3 -u bench.py --config 1 --kind local --gap-open -2 --no-cpu-baseline > $OUT/al_${t}_$i.json 2> $OUT/al_${t}_$i.err
  done
done
echo done
