#!/bin/bash
# A/B of library variants on the throughput-bound genome workloads: configs[4] N=1 (score,
# twice each) and configs[3] (construct, once each).  Usage: ab34.sh <tag> <variants>
set -o pipefail
TAG=$1; VS=$2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  local libenv=""
  [ "$lib" != prod ] && libenv="ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_$lib.so"
  env $libenv timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-anchor --kernel-steps 1 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);print('$name', d['value'], d['ms_per_step'], d['config'].get('score'), d['config'].get('result_check',{}).get('checked'))"
}
for i in 1 2; do
  for V in ${VS//,/ }; do
    run c4_${V}_$i $V --config 4 --steps 1 --warmup 1
  done
done
for V in ${VS//,/ }; do
  run c3_${V} $V --config 3 --steps 1 --warmup 1
done
echo DONE
