set -o pipefail
O=gpurun_out/r06w_tr
mkdir -p $O
export TMPDIR=/tmp
for V in 1 0; do
  ANYSEQ_AFFINE_TRANSPOSE=$V timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-anchor --kernel-steps 1 --config 3 --steps 1 --warmup 1 > $O/c3_t$V.json 2> $O/c3_t$V.err || { echo FAIL $V; tail -5 $O/c3_t$V.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/c3_t$V.json') if l.startswith('{')][-1]);print('t$V', d['value'], d['ms_per_step'], d['config'].get('fill_gcups'), d['config'].get('result_check',{}).get('checked'))"
done
