#!/bin/bash
# the whole GPU parity suite (with the loaded-library record), smoke(), one bench line
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
ANYSEQ_MAPS_OUT=$O/loaded_libs.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt | tail -2
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][-1]);print(d['value'], d['config']['result_check'], d['roofline']['chain_model']['cycles_per_chain_step'], d.get('scaling_anchor',{}).get('value'))"
