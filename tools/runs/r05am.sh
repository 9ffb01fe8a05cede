#!/bin/bash
# Round 5: the I/O wave on the first hardware wave (shares its SIMD with the group's last band): parity, A/B.
set -o pipefail
O=gpurun_out/r05am; mkdir -p $O
ANYSEQ_IO_FIRST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_linear_affine.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for rep in 1 2; do
for v in 0 1; do
ANYSEQ_IO_FIRST=$v timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-anchor > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
ANYSEQ_IO_FIRST=$v timeout -k 10 200 python -u bench.py --config 1 --kind local --gap-open -2 --steps 6 --warmup 2 --no-cpu-baseline > $O/al_${v}_$rep.json 2> $O/al_${v}_$rep.err || { tail -20 $O/al_${v}_$rep.err; exit 1; }
ANYSEQ_IO_FIRST=$v timeout -k 10 200 python -u bench.py --config 1 --steps 6 --warmup 2 --no-cpu-baseline > $O/c1_${v}_$rep.json 2> $O/c1_${v}_$rep.err || { tail -20 $O/c1_${v}_$rep.err; exit 1; }
done
done
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d.get('ms_per_step_min'))"; done
