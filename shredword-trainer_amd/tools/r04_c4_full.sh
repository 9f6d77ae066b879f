#!/bin/bash
# Round-4: C4 at full size (80 GB UTF-8, vocab 32000, mpf 2000, the 8-range sharded load counted in
# turn) on one GPU, with the load phases and the resident loop's per-launch report.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_LOAD_REPORT=1 SHREDWORD_RESIDENT_REPORT=1 SHREDWORD_ENGINE_REPORT=1 timeout -k 10 1100 python -u \
  shredword-trainer_amd/tools/fullsize_run.py --config c4 --known profiles/r03_c4_80g_fullsize.json \
  --out gpurun_out/r04_c4_80g_full.json > gpurun_out/r04_c4_80g_full.log 2>&1
