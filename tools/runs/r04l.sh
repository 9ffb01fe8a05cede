#!/bin/bash
# Round 4: asynchronous subject staging, chunked final-level sweep reads -- parity, configs[2], affine local
# score, configs[4] at N=1, band timeline (stamps build).
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl.json 2> $O/afl.err || exit 1
timeout -k 10 300 $B --config 4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
timeout -k 10 60 tools/micro/bin/pw_micro > $O/pw_micro.txt 2>&1 || exit 1
