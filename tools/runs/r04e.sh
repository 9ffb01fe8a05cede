#!/bin/bash
# Round 4: affine waves per workgroup chosen per launch (NWA auto): parity + configs[2]/[3]/[4].
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py \
  tests/test_gpu_shard_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 200 $B --config 4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 $B --config 3 --steps 1 --warmup 1 > $O/c3.json 2> $O/c3.err || exit 1
