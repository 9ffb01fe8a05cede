mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_affine_construct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_affc.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_affc.log | head -40
tail -3 gpurun_out/pytest_affc.log
exit $rc
