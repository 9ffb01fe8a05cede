#!/bin/bash
# Round 4: latency micros, band timeline (stamps build), kernel trace of configs[2].
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
for b in isa_micro pingpong_micro lat_micro step_lat aff_micro; do
  timeout -k 10 60 tools/micro/bin/$b > $O/$b.txt 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/probes/_aff_timeline.py $O/tl > $O/timeline.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 -- python3 bench.py --no-cpu-baseline --no-anchor --steps 4 --warmup 1 > $O/prof_c2.json 2> $O/prof_c2.err || exit 1
