#!/bin/bash
# Round-4 GPU check 2: the one-card rehearsal of the N=2 one-training bench (ranks share the GPU,
# word lists over gloo), then the C5 and C4 parameters at 10 GB as full bench lines (K1 leg, CPU
# baseline, parity against the c5_10g / c4_10g oracle runs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_LOAD_REPORT=1 timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 > gpurun_out/r04_c3_2ranks_one_gpu.json 2> gpurun_out/r04_c3_2ranks_one_gpu.err || exit $?
SHREDWORD_LOAD_REPORT=1 timeout -k 10 600 python bench.py --config c5 --bytes 10000000000 --steps 3 --warmup 1 \
  --pair-count-reps 5 --encode-reps 3 > gpurun_out/r04_c5_10g_bench.json 2> gpurun_out/r04_c5_10g_bench.err || exit $?
