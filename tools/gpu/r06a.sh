#!/bin/bash
# round 6, first GPU pass: the new parity tests, the construct fixture of configs[3], a bench line
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_true_construct.py tests/test_gpu_shard_hostcoll.py \
    tests/test_gpu_rccl_ranks.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-anchor > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
timeout -k 10 300 python -u tests/golden/make_config4_fixture.py --construct > $O/fixture.log 2>&1 || { tail -20 $O/fixture.log; exit 1; }
cp tests/golden/config4_synthetic.json $O/
echo DONE
