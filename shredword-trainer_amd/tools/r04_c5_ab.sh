#!/bin/bash
# Round-4: C5 100 GB, one load, the final defaults against the opt-in host pipelining.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_ENGINE_REPORT=1 timeout -k 10 1100 python -u shredword-trainer_amd/tools/option_sweep.py --config c5 \
  --set - early_guess=1,apply_helper=1 early_guess=1 - --out gpurun_out/r04_c5_option_ab.json \
  > gpurun_out/r04_c5_option_ab.log 2>&1
