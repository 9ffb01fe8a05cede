#!/bin/bash
# Round 5: device-planned round-robin levels of the sharded construct (item 6): the
# sharded construct suites (emulated ranks), the RCCL worker test, the single-GPU
# construct suites, one configs[2] bench line.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
T="timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu"
$T tests/test_gpu_shard_construct.py > $O/pytest_shard_construct.log 2>&1 || exit 1
$T tests/test_gpu_rccl_ranks.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_golden.py > $O/pytest_rest.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-anchor --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
tail -3 $O/pytest_shard_construct.log; tail -3 $O/pytest_rest.log; cat $O/c2.json
