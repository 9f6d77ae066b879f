#!/bin/bash
# Round-4 GPU check 11: tiebreak=device with the smaller, growing pair table (tests + C3 line).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiebreak.py -v --timeout 240 --timeout-method thread \
  > gpurun_out/r04_tiebreak_tests3.log 2>&1 || exit $?
SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device --steps 3 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_device5.json 2> gpurun_out/r04_c3_device5.err || exit $?
