#!/bin/bash
# parity subset on an experimental library (short limits).  Usage: exp_check.sh <tag> <lib> tests...
set -o pipefail
O=gpurun_out/$1; L=$2; shift 2
mkdir -p $O
export TMPDIR=/tmp
ANYSEQ_LIB=$PWD/anyseq_amd/libanyseq_$L.so timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/pytest_$L.log 2>&1 || { tail -30 $O/pytest_$L.log; exit 1; }
tail -2 $O/pytest_$L.log
