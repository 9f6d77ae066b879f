#!/bin/bash
# Round-4 GPU check 3: C4's parameters at 10 GB through the 8-range sharded load as a full bench
# line (parity against the c4_10g oracle run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_LOAD_REPORT=1 timeout -k 10 600 python bench.py --config c4 --bytes 10000000000 --steps 3 --warmup 1 \
  --pair-count-reps 5 --encode-reps 3 > gpurun_out/r04_c4_10g_bench.json 2> gpurun_out/r04_c4_10g_bench.err || exit $?
