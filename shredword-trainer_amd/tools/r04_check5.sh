#!/bin/bash
# Round-4 GPU check 5: the 2-rank one-card rehearsal again (range tables sized by the file), the
# device-mode C3 line, then C5 at full size (100 GB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_LOAD_REPORT=1 timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 > gpurun_out/r04_c3_2ranks_c.json 2> gpurun_out/r04_c3_2ranks_c.err || exit $?
bash shredword-trainer_amd/tools/r04_c5_full.sh
