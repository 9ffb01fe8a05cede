#!/bin/bash
# Round 5: two rows per lane (affine_rows_per_lane 2) parity, then the one-row affine suite.
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_affine_r2.py > $O/r2.log 2>&1 || { tail -40 $O/r2.log; exit 1; }
tail -3 $O/r2.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine.py tests/test_gpu_shard_affine.py > $O/aff.log 2>&1 || { tail -40 $O/aff.log; exit 1; }
tail -3 $O/aff.log
