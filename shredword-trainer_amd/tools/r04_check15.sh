#!/bin/bash
# Round-4 GPU check 15: the early guess bounded by the merge's record count, at C3 (A/B) and C4 80 GB.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=2 STEPS=5 TAG=_earlymax bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_EARLY_GUESS=0" "SHREDWORD_EARLY_MAX_RECORDS=150" "X=1" || exit $?
SHREDWORD_ENGINE_REPORT=1 timeout -k 10 1000 python -u shredword-trainer_amd/tools/option_sweep.py --config c4 \
  --set - early_guess=0 early_max_records=150 early_max_records=300 - --out gpurun_out/r04_c4_early_ab.json \
  > gpurun_out/r04_c4_early_ab.log 2>&1
