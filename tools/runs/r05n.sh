#!/bin/bash
# Round 5: band timeline with the light stamps (steady start/end only: product-like step)
# and the clock per band; the full stamps build beside it.
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
ANYSEQ_TL_LIB=anyseq_amd/libanyseq_stamps_light.so timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tll > $O/timeline_light.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
