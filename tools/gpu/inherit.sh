#!/bin/bash
# inherited halves: parity suite, the genome-length construct fixture,
# then configs[3] with the option on / off (and the transposition knob)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inherit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_inherit.txt 2>&1 || { tail -40 $O/pytest_inherit.txt; exit 1; }
tail -3 $O/pytest_inherit.txt
ANYSEQ_INHERIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_golden_affine.py tests/test_gpu_affine_construct.py -x -v --timeout 300 --timeout-method thread > $O/pytest_affc.txt 2>&1 || { tail -40 $O/pytest_affc.txt; exit 1; }
tail -3 $O/pytest_affc.txt
for V in 1 0; do
  ANYSEQ_INHERIT=$V timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-anchor --kernel-steps 1 --config 3 --steps 1 --warmup 1 > $O/c3_i$V.json 2> $O/c3_i$V.err || { echo FAIL $V; tail -5 $O/c3_i$V.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/c3_i$V.json') if l.startswith('{')][-1]);print('inherit $V', d['value'], d['ms_per_step'], d['config'].get('fill_gcups'), d['config'].get('fill_launches_per_step'), d['config'].get('result_check',{}).get('checked'))"
done
