#!/bin/bash
# Fill time vs query length (m fixed): separates the per-band lag from the per-step time.
OUT=gpurun_out/shape_$1
mkdir -p $OUT
: > $OUT/results.jsonl
for C in "--config 1" "--config 1 --kind local --gap-open -2" "--config 1 --kind global --gap-open -2"; do
  for N in 512 2048 8192 32768 65536; do
    echo "[shape] $C n=$N" >&2
    timeout -k 10 120 python3 bench.py $C --n $N --steps 5 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2> $OUT/err.txt || { tail -3 $OUT/err.txt; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1])
print(json.dumps({'cfg':'$C','n':$N,'kernel_ms':d['roofline']['kernel_ms'],'value':d['value']}))" >> $OUT/results.jsonl
  done
done
cat $OUT/results.jsonl
