#!/bin/bash
# Round 5: bench steps without per-launch fill events (kernels timed in a separate pass):
# parity of the event-free path, configs[2] / [1] / affine local lines, kernel trace gaps.
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
$T tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_a.json 2> $O/c2_a.err || exit 1
timeout -k 10 120 $B --config 1 --steps 10 --warmup 3 > $O/c1.json 2> $O/c1.err || exit 1
timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl.json 2> $O/afl.err || exit 1
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_b.json 2> $O/c2_b.err || exit 1
ANYSEQ_FILL_EVENTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-anchor --kernel-steps 1 > $O/trace.log 2>&1 || exit 1
tail -2 $O/pytest.log; for f in c2_a c1 afl c2_b; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_timing']['steps'])"; done
