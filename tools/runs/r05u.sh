#!/bin/bash
# Round 5: one combined scan in the level plan, wave-summed cells, four-stream descriptor
# digest: construct parity (single GPU and sharded), tail phases, configs[2] bench.
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
T="timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
$T tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_golden.py tests/test_gpu_shard_construct.py tests/test_gpu_fault_regression.py > $O/pytest.log 2>&1 || exit 1
ANYSEQ_TAIL_STAMPS=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-anchor --steps 2 --warmup 1 > $O/c2_st.json 2> $O/c2_st.err || exit 1
timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-anchor --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
tail -2 $O/pytest.log; tail -9 $O/c2_st.err; grep -o '"value": [0-9.]*' $O/c2.json; grep -o '"nonfill_ms": [0-9.]*' $O/c2.json
