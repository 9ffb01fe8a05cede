#!/bin/bash
# GPU box: the GPU suite, then configs[4] N=1 and configs[2] lines.  Usage: bash tools/gpu_r03g.sh
set -e
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err
timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-anchor > $OUT/c2.json 2> $OUT/c2.err
echo done
