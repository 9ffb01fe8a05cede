#!/bin/bash
# GPU box: linear fill bench (I/O wave A/B), the GPU suite, configs[3] / configs[4] N=1 lines.
# Usage (repo root, on the box): bash tools/gpu_r03f.sh
set -e
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --config 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c1_$i.json 2> $OUT/c1_$i.err
done
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 300 python3 -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err
echo done
