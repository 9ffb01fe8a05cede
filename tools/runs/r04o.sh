#!/bin/bash
# Round 4: A/B of the affine I/O wave's subject staging modes (ANYSEQ_IO_STAGE 0..3) on one
# box, interleaved; final-level micro; parity on the default mode.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 60 tools/micro/bin/pw_micro > $O/pw_micro.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2; do
  for m in 0 1 2 3; do
    ANYSEQ_IO_STAGE=$m timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_m${m}_r$rep.json 2> $O/c2_m${m}_r$rep.err || exit 1
    ANYSEQ_IO_STAGE=$m timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_m${m}_r$rep.json 2> $O/afl_m${m}_r$rep.err || exit 1
  done
done
