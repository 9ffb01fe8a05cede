#!/bin/bash
# Round 5: hand-off polls spinning instead of s_sleep 1 (libanyseq_exp.so: ANYSEQ_GEN_SLEEP=0)
# and the forwarder's hand-off step at issue priority 3 (ANYSEQ_PRIO=3), A/B on one box;
# the chain probe for the default and the spinning build.
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
EXP=$PWD/anyseq_amd/libanyseq_exp.so
ANYSEQ_LIB=$EXP timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_affine.py > $O/pytest_exp.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-anchor"
AFL="--config 1 --kind local --gap-open -2"
for rep in 1 2; do
  timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_def_r$rep.json 2> $O/c2_def_r$rep.err || exit 1
  timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_def_r$rep.json 2> $O/afl_def_r$rep.err || exit 1
  ANYSEQ_LIB=$EXP timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_spin_r$rep.json 2> $O/c2_spin_r$rep.err || exit 1
  ANYSEQ_LIB=$EXP timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_spin_r$rep.json 2> $O/afl_spin_r$rep.err || exit 1
  ANYSEQ_PRIO=3 timeout -k 10 120 $B --steps 10 --warmup 3 > $O/c2_prio3_r$rep.json 2> $O/c2_prio3_r$rep.err || exit 1
  ANYSEQ_PRIO=3 timeout -k 10 120 $B $AFL --steps 10 --warmup 3 > $O/afl_prio3_r$rep.json 2> $O/afl_prio3_r$rep.err || exit 1
done
timeout -k 10 300 python -u tools/probes/_chain_probe.py 3 > $O/chain_def.txt 2>&1 || exit 1
ANYSEQ_LIB=$EXP timeout -k 10 300 python -u tools/probes/_chain_probe.py 3 > $O/chain_spin.txt 2>&1 || exit 1
