#!/bin/bash
# One GPU-box pass: the GPU parity suite, then the round profile (bench lines,
# rocprof stats, PMC passes).  Usage (repo root, on the box): bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
tail -n 1 gpurun_out/pytest_$TAG.log
bash tools/profile.sh $TAG
