#!/bin/bash
# Round 4: A/B of two hand-off polls in flight in the affine I/O wave (ANYSEQ_IO_POLL2 0/1),
# interleaved on one box, with parity of the affine suite under 1.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
ANYSEQ_IO_POLL2=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
for rep in 1 2 3; do
  for p2 in 0 1; do
    ANYSEQ_IO_POLL2=$p2 timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_p${p2}_r$rep.json 2> $O/c2_p${p2}_r$rep.err || exit 1
    ANYSEQ_IO_POLL2=$p2 timeout -k 10 120 $B --config 1 --kind local --gap-open -2 --steps 10 --warmup 3 > $O/afl_p${p2}_r$rep.json 2> $O/afl_p${p2}_r$rep.err || exit 1
  done
done
ANYSEQ_IO_POLL2=1 timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
