#!/bin/bash
# One GPU-box pass: parity tests, then the round profile (bench + rocprof stats + PMC).
# Usage (from the repo root, on the box): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -e
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${2:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
bash tools/profile.sh $TAG
