#!/bin/bash
# Round profile collection on the GPU box (repo root): bench lines, kernel-trace
# stats, PMC passes (HBM bytes and SQ counters), for the default workload
# (configs[2]), configs[1] and configs[4] at N=1.  Every step has its own time limit; the first
# failure ends the script.
# Usage: bash tools/profile.sh <tag>
set -e
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
run() {   # run <name> <timeout> <cmd...>: stdout to $OUT/<name>.json, stderr to $OUT/<name>.err
    local name=$1 t=$2
    shift 2
    echo "[profile] $name" >&2
    timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err
}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
run bench 300 python3 bench.py
run bench_c1 300 python3 bench.py --config 1
run bench_aff_local 300 python3 bench.py --config 1 --kind local --gap-open -2 --no-cpu-baseline
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B
run fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B
run write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B
run sq 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq -o run -- $B
B1="python3 bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline"
run trace_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o run -- $B1
run fetch_c1 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_c1 -o run -- $B1
run write_c1 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_c1 -o run -- $B1
run sq_c1 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq_c1 -o run -- $B1
B2="python3 bench.py --config 1 --kind local --gap-open -2 --steps 3 --warmup 1 --no-cpu-baseline"
run sq_aff_local 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq_aff_local -o run -- $B2
run trace_aff_local 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_aff_local -o run -- $B2
# configs[4] at N=1 (throughput-bound: two rows per lane, round 5)
B4="python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline"
run bench_c4 300 $B4
run trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -o run -- $B4
run sq_c4 200 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq_c4 -o run -- $B4
echo "[profile] done" >&2
