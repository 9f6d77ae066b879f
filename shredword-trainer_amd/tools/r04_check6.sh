#!/bin/bash
# Round-4 GPU check 6: the profiles (kernel trace + stats, PMC passes, engine trace), then the
# 2-rank one-card rehearsal with the gather / merge timings.
set -o pipefail
bash shredword-trainer_amd/tools/r04_prof.sh || exit $?
SHREDWORD_LOAD_REPORT=1 timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 > gpurun_out/r04_c3_2ranks_d.json 2> gpurun_out/r04_c3_2ranks_d.err || exit $?
SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device --steps 2 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_device3.json 2> gpurun_out/r04_c3_device3.err || exit $?
