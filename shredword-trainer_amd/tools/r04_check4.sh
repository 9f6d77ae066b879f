#!/bin/bash
# Round-4 GPU check 4: tiebreak=device with its early merges on the whole-chip resident loop (host
# selection by the same rule), the tests and a C3 line with the per-launch report; the one-card
# 2-rank rehearsal with the load's repeat reasons; then C5 at full size (100 GB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiebreak.py -v --timeout 240 --timeout-method thread \
  > gpurun_out/r04_tiebreak_tests.log 2>&1 || exit $?
SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device --steps 3 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_device2.json 2> gpurun_out/r04_c3_device2.err || exit $?
SHREDWORD_LOAD_REPORT=1 timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 2 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 > gpurun_out/r04_c3_2ranks_b.json 2> gpurun_out/r04_c3_2ranks_b.err || exit $?
bash shredword-trainer_amd/tools/r04_c5_full.sh
