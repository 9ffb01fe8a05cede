#!/bin/bash
# Round 5: the forwarder I/O wave (io_forward) against the full io_wave with code rows
# (ANYSEQ_IO_FWD=0), A/B on one box; band timeline of the default (stamps build).
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_affine.py > $O/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
for rep in 1 2; do
  for f in 1 0; do
    ANYSEQ_IO_FWD=$f timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_f${f}_r$rep.json 2> $O/c2_f${f}_r$rep.err || exit 1
    ANYSEQ_IO_FWD=$f timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_f${f}_r$rep.json 2> $O/afl_f${f}_r$rep.err || exit 1
  done
done
timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
