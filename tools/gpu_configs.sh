#!/bin/bash
# GPU box: parity tests, then bench lines of configs[1..3] + rocprof stats of configs[2].
# Usage (on the box, repo root): bash tools/gpu_configs.sh <tag>
set -e
TAG=${1:-r01d}
OUT=gpurun_out/cfg_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py > $OUT/bench_c1.json 2> $OUT/bench_c1.err
timeout -k 10 300 python bench.py --config 2 --steps 3 --warmup 1 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2 -o run -- python3 bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c2_trace.json 2> $OUT/trace_c2.err
timeout -k 10 500 python -u bench.py --config 3 --steps 1 --warmup 0 > $OUT/bench_c3.json 2> $OUT/bench_c3.err
cat $OUT/bench_c1.json $OUT/bench_c2.json $OUT/bench_c3.json
