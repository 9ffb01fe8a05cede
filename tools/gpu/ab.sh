#!/bin/bash
# A/B of library builds / tuning variants on one box: bench lines (configs[2], the affine
# local score) interleaved, twice each.  Usage: bash tools/gpu/ab.sh <tag> <variant>...
# variant: <lib>[:ENV=V[,ENV=V...]] with lib "prod" or a suffix X of anyseq_amd/libanyseq_X.so
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --kernel-steps 1"
run() {  # name variant args...
  local name=$1 var=$2; shift 2
  local lib=${var%%:*} envs=""
  [[ "$var" == *:* ]] && envs=${var#*:}
  local libenv=""
  [ "$lib" != prod ] && libenv="ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_$lib.so"
  env $libenv ${envs//,/ } timeout -k 10 240 $B "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]);print('$name', '$var', d['value'], d['config'].get('score'), d['config'].get('fill_ms_per_step'), d['roofline'].get('chain_model',{}).get('cycles_per_chain_step'))"
}
for i in 1 2; do
  j=0
  for V in "$@"; do
    j=$((j+1))
    run c2_v${j}_$i "$V"
    run loc_v${j}_$i "$V" --config 1 --kind local --gap-open -2
  done
done
echo DONE
