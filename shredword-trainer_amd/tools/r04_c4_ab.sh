#!/bin/bash
# Round-4: C4 80 GB, one load, the engine options A/B'd (early guess, apply helper).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_ENGINE_REPORT=1 timeout -k 10 1100 python -u shredword-trainer_amd/tools/option_sweep.py --config c4 \
  --set - early_guess=0 apply_helper=0 early_guess=0,apply_helper=0 - --out gpurun_out/r04_c4_option_ab.json \
  > gpurun_out/r04_c4_option_ab.log 2>&1
