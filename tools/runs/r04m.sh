#!/bin/bash
# Round 4: final level -- uniform wave index in the sweep, branch-free scalar walk: micro,
# parity (construct, golden, shard construct), configs[2] with a kernel trace.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 60 tools/micro/bin/pw_micro > $O/pw_micro.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_shard_construct.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- python3 bench.py --no-cpu-baseline --no-anchor --steps 4 --warmup 1 > $O/prof_c2.json 2> $O/prof_c2.err || exit 1
