#!/bin/bash
# Round 5: XCD-local groups (ANYSEQ_XCD_GROUPS / xcd_groups): parity (its own test, the
# affine construct tests and the configs[2] fixtures with the option on), then A/B on one
# box against the single queue (affine local score, configs[2]), and io_skew 16 / 32.
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
$T tests/test_gpu_affine.py -k "xcd or fused or positive" > $O/pytest_xcd_test.log 2>&1 || exit 1
ANYSEQ_XCD_GROUPS=1 $T tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_affine.py > $O/pytest_xcd.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
for rep in 1 2; do
  for x in 0 1; do
    ANYSEQ_XCD_GROUPS=$x timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_x${x}_r$rep.json 2> $O/c2_x${x}_r$rep.err || exit 1
    ANYSEQ_XCD_GROUPS=$x timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_x${x}_r$rep.json 2> $O/afl_x${x}_r$rep.err || exit 1
  done
  for k in 16 32; do
    ANYSEQ_IO_SKEW=$k timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_skew${k}_r$rep.json 2> $O/afl_skew${k}_r$rep.err || exit 1
  done
done
