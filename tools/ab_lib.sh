set -e
mkdir -p gpurun_out/ab
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-anchor"
for i in 1 2; do
  for L in libanyseq.so libanyseq_prev.so; do
    ANYSEQ_LIB=$PWD/anyseq_amd/$L timeout -k 10 120 $B --config 1 --kind local --gap-open -2 > gpurun_out/ab/aff_${L}_$i.json 2>gpurun_out/ab/aff_${L}_$i.err
    ANYSEQ_LIB=$PWD/anyseq_amd/$L timeout -k 10 120 $B > gpurun_out/ab/c2_${L}_$i.json 2>gpurun_out/ab/c2_${L}_$i.err
  done
done
echo done
