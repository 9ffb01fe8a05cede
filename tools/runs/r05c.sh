#!/bin/bash
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u tools/probes/_posmis_probe.py > $O/probe.log 2>&1 || exit 1
