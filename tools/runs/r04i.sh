#!/bin/bash
# Round 4: the whole GPU suite on the current build, then r04f's measurements.
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
bash tools/runs/r04f.sh
