#!/bin/bash
# Round 4: sharded construct over rank subgroups + adaptive chunks (GPU parity), then r04f's measurements.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_shard_construct.py tests/test_gpu_shard_affine.py tests/test_gpu_shard.py > $O/pytest.log 2>&1 || exit 1
bash tools/runs/r04f.sh
