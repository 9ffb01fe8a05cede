set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_shard.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_shard.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 ; rc=$?
tail -3 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --sharded > gpurun_out/bench_sharded1.json 2> gpurun_out/bench_sharded1.err; rc=$?
cat gpurun_out/bench_sharded1.json; tail -3 gpurun_out/bench_sharded1.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err; cat gpurun_out/bench1.json
