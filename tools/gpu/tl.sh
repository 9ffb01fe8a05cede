#!/bin/bash
# band timelines (light stamps builds) of the 65536^2 affine local score
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
export TMPDIR=/tmp
for L in "$@"; do
  ANYSEQ_TL_LIB=anyseq_amd/libanyseq_$L.so timeout -k 10 200 python3 -u tools/aff_timeline.py $O/tl_$L > $O/tl_$L.log 2>&1 || { tail -20 $O/tl_$L.log; exit 1; }
  echo "== $L"; cat $O/tl_$L.log
done
