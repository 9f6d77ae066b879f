#!/bin/bash
# Round-4 GPU check 16: the 4-rank one-card rehearsal of the replicate bench (world 4, one C3
# training, bit-exact against the oracle's full run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHREDWORD_LOAD_REPORT=1 timeout -k 10 600 python bench.py --gpus 4 --config c3 --steps 1 --warmup 0 --encode-reps 0 \
  --pair-count-reps 0 > gpurun_out/r04_c3_4ranks_one_gpu.json 2> gpurun_out/r04_c3_4ranks_one_gpu.err || exit $?
