#!/bin/bash
# Bench lines under tuning environment variants (GPU box, repo root).
# Usage: bash tools/sweep_env.sh <tag> "<ENV=V ...>" ... ; each variant runs configs 1, 1-affine-local, 2.
TAG=$1
shift
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
i=0
for VARS in "$@"; do
    i=$((i+1))
    for C in "--config 1" "--config 1 --kind local --gap-open -2" "--config 2"; do
        echo "[sweep] $VARS :: $C" >&2
        env $VARS timeout -k 10 120 python3 bench.py $C --steps 5 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2> $OUT/err_$i.txt || exit 1
        python3 -c "
import json,sys
d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1])
print(json.dumps({'vars':'$VARS','cfg':'$C','value':d['value'],'ms':d['ms_per_step_median'],'kernel_ms':d['roofline']['kernel_ms'],'score':d['config']['score']}))" >> $OUT/results.jsonl
    done
done
cat $OUT/results.jsonl
