#!/bin/bash
# Round 5: the GS kernel without io_wave (no call, no scratch): affine parity, configs[2]
# bench, kernel trace of a short run (launch gaps around the fills).
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
$T tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest_aff.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_a.json 2> $O/c2_a.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-anchor > $O/trace.log 2>&1 || exit 1
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_b.json 2> $O/c2_b.err || exit 1
tail -2 $O/pytest_aff.log; grep -o '"value": [0-9.]*' $O/c2_a.json $O/c2_b.json
