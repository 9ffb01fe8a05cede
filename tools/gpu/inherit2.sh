#!/bin/bash
# inherited halves, recorded depth: parity suite (depths 1-3), the genome-length fixtures with
# the default, configs[3] at depth 1 / 2 / 3
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inherit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_inherit.txt 2>&1 || { tail -40 $O/pytest_inherit.txt; exit 1; }
tail -3 $O/pytest_inherit.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden_affine.py -x -v --timeout 300 --timeout-method thread > $O/pytest_golden.txt 2>&1 || { tail -40 $O/pytest_golden.txt; exit 1; }
tail -3 $O/pytest_golden.txt
for D in 1 2 3; do
  ANYSEQ_INHERIT_DEPTH=$D timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-anchor --kernel-steps 1 --config 3 --steps 1 --warmup 1 > $O/c3_d$D.json 2> $O/c3_d$D.err || { echo FAIL $D; tail -5 $O/c3_d$D.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/c3_d$D.json') if l.startswith('{')][-1]);print('depth $D', d['value'], d['ms_per_step'], d['config'].get('fill_gcups'), d['config'].get('fill_cells_per_step'), d['config'].get('fill_launches_per_step'), d['config'].get('result_check',{}).get('checked'))"
done
