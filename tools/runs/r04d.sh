#!/bin/bash
# Round 4: production-loop micro with the "st" hand-off, its parity, and an A/B (ANYSEQ_AFF_PUB 0 / 1).
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 120 tools/micro/bin/aff_loop_micro > $O/aff_loop_micro.txt 2>&1 || exit 1
ANYSEQ_AFF_PUB=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py \
  tests/test_gpu_shard_construct.py tests/test_gpu_shard_affine.py > $O/pytest_pub1.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for pub in 0 1; do
  ANYSEQ_AFF_PUB=$pub timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_pub$pub.json 2> $O/c2_pub$pub.err || exit 1
  ANYSEQ_AFF_PUB=$pub timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_pub$pub.json 2> $O/afl_pub$pub.err || exit 1
done
