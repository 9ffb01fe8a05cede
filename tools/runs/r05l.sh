#!/bin/bash
# Round 5: the product build's band chain measured from outside (fill time against the
# number of bands per front, tools/probes/_chain_probe.py); the loop micro on this build.
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u tools/probes/_chain_probe.py 3 > $O/chain.txt 2>&1 || exit 1
