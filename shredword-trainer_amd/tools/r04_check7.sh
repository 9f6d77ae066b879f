#!/bin/bash
# Round-4 GPU check 7: tiebreak=device tests and C3 line after the compaction policy change, then
# the C5 100 GB hybrid switch sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiebreak.py -v --timeout 240 --timeout-method thread \
  > gpurun_out/r04_tiebreak_tests2.log 2>&1 || exit $?
SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device --steps 3 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_device4.json 2> gpurun_out/r04_c3_device4.err || exit $?
SHREDWORD_RESIDENT_REPORT=1 timeout -k 10 800 python -u shredword-trainer_amd/tools/c5_switch_sweep.py \
  --occ 4000 12000 40000 --out gpurun_out/r04_c5_switch_sweep.json > gpurun_out/r04_c5_switch_sweep.log 2>&1
