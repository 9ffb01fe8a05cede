#!/bin/bash
# Round 5: the quarter publisher (PUB8: lane 63 stores its own cells, no DPP shift
# register).  Loop micro, parity (affine suites, golden, shards), A/B against the shift
# register (libanyseq_exp.so: ANYSEQ_GEN_PUB8=0) on configs[2], affine local score,
# configs[4]-shaped throughput (semiglobal affine score 1048576 x 1048576).
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 120 tools/micro/bin/mix_micro_lds > $O/mix_lds.txt 2>&1 || exit 1
timeout -k 10 120 tools/micro/bin/mix_micro_llds > $O/mix_llds.txt 2>&1 || exit 1
T="timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
$T tests/test_gpu_affine.py tests/test_gpu_affine_construct.py tests/test_gpu_golden_affine.py tests/test_gpu_golden.py > $O/pytest_aff.log 2>&1 || exit 1
$T tests/test_gpu_shard_affine.py tests/test_gpu_shard_construct.py tests/test_gpu_fault_regression.py > $O/pytest_shard.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
SG="--config 1 --kind semiglobal --gap-open -2 --n 1048576 --m 1048576"
for rep in 1 2; do
  for lib in libanyseq.so libanyseq_exp.so; do
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_${lib%.so}_r$rep.json 2> $O/c2_${lib%.so}_r$rep.err || exit 1
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_${lib%.so}_r$rep.json 2> $O/afl_${lib%.so}_r$rep.err || exit 1
    ANYSEQ_LIB=$PWD/anyseq_amd/$lib timeout -k 10 120 $B $SG --steps 3 --warmup 1 > $O/sg_${lib%.so}_r$rep.json 2> $O/sg_${lib%.so}_r$rep.err || exit 1
  done
done
cat $O/mix_lds.txt $O/mix_llds.txt | grep "FULL\|VALU "
grep -h '"value"' $O/*.json | python3 -c "
import sys, json
for l in sys.stdin: pass
" ; for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('ms_per_step'))")"; done
