#!/bin/bash
# Round-4: C5 at full size (100 GB mixed script, vocab 64000, coverage 0.9995) on one GPU, with the
# load phase report: the streamed load against round 3's 19-23 s, the same .model/.vocab md5 as the
# round-3 run of the same corpus (profiles/r03_c5_100g_fullsize.json).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
SHREDWORD_LOAD_REPORT=1 SHREDWORD_RESIDENT_REPORT=1 timeout -k 10 1100 python -u shredword-trainer_amd/tools/fullsize_run.py \
  --config c5 --known profiles/r03_c5_100g_fullsize.json --out gpurun_out/r04_c5_100g_full.json \
  > gpurun_out/r04_c5_100g_full.log 2>&1
