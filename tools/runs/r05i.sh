#!/bin/bash
# Round 5: subject codes from HBM code rows (GS, the default build) -- the I/O wave only
# forwards hand-off rows.  Parity (affine suites, golden fixtures, shard paths), A/B on one
# box against the round-4 LDS subject path (libanyseq_exp.so: GS=0), band timeline.
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
$T tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_golden.py > $O/pytest_aff.log 2>&1 || exit 1
$T tests/test_gpu_shard_affine.py tests/test_gpu_shard_construct.py tests/test_gpu_fault_regression.py > $O/pytest_shard.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
for rep in 1 2; do
  for lib in libanyseq.so libanyseq_exp.so; do
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_${lib%.so}_r$rep.json 2> $O/c2_${lib%.so}_r$rep.err || exit 1
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_${lib%.so}_r$rep.json 2> $O/afl_${lib%.so}_r$rep.err || exit 1
  done
done
timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
