#!/bin/bash
# A/B of the affine fill's compute waves per workgroup (ANYSEQ_NWA 4 vs 7), round 4.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 120 tools/micro/bin/aff_loop_micro > $O/aff_loop_micro.txt 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline"
for nw in 4 7; do
  ANYSEQ_NWA=$nw timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_nw$nw.json 2> $O/c2_nw$nw.err || exit 1
  ANYSEQ_NWA=$nw timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_nw$nw.json 2> $O/afl_nw$nw.err || exit 1
done
for nw in 4 7; do
  ANYSEQ_NWA=$nw timeout -k 10 200 $B --config 4 --steps 2 --warmup 1 > $O/c4_nw$nw.json 2> $O/c4_nw$nw.err || exit 1
done
ANYSEQ_NWA=7 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest_nw7.log 2>&1 || exit 1
timeout -k 10 120 tools/micro/bin/aff_loop_micro > $O/aff_loop_micro.txt 2>&1 || exit 1
