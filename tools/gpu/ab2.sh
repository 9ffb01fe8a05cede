#!/bin/bash
# A/B of library variants on one box without the result gate's construct line for
# diagnostic builds.  Usage: bash tools/gpu/ab2.sh <tag> <c2-variants> <loc-only-variants>
# (comma-separated lists; "prod" or a suffix X of anyseq_amd/libanyseq_X.so)
set -o pipefail
TAG=$1; C2=$2; LOC=$3
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --kernel-steps 1"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  local libenv=""
  [ "$lib" != prod ] && libenv="ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_$lib.so"
  env $libenv timeout -k 10 240 $B "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);print('$name', d['value'], d['config'].get('score'), d['config'].get('fill_ms_per_step'), d['roofline'].get('chain_model',{}).get('cycles_per_chain_step'))"
}
for i in 1 2; do
  for V in ${C2//,/ }; do
    run c2_${V}_$i $V
    run loc_${V}_$i $V --config 1 --kind local --gap-open -2
  done
  for V in ${LOC//,/ }; do
    run loc_${V}_$i $V --config 1 --kind local --gap-open -2
  done
done
echo DONE
