#!/bin/bash
# GPU box: full parity suite, then the fill timing probe with the I/O wave generating
# band 0's top border (default) and with band 0 writing it itself.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_iob.log 2>&1
tail -2 gpurun_out/gpu_iob.log
ANYSEQ_IO_BORDER=1 timeout -k 10 200 python -u tools/perf_probe.py > gpurun_out/perf_iob1.log 2>&1
ANYSEQ_IO_BORDER=0 timeout -k 10 200 python -u tools/perf_probe.py > gpurun_out/perf_iob0.log 2>&1
ANYSEQ_IO_BORDER=1 timeout -k 10 200 python -u tools/perf_probe.py > gpurun_out/perf_iob1b.log 2>&1
head -6 gpurun_out/perf_iob1.log gpurun_out/perf_iob0.log gpurun_out/perf_iob1b.log
