#!/bin/bash
# configs[1] bench lines under tuning environment variants (GPU box, repo root).
TAG=$1
shift
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
for VARS in "$@"; do
    echo "[sweep] $VARS" >&2
    env $VARS timeout -k 10 120 python3 bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1])
print(json.dumps({'vars':'$VARS','value':d['value'],'ms':d['ms_per_step_median'],'kernel_ms':d['roofline']['kernel_ms'],'score':d['config']['score']}))" >> $OUT/results.jsonl
done
cat $OUT/results.jsonl
