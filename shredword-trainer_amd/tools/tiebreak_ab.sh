#!/bin/bash
# tiebreak=device against the exact mode on one box: test_gpu_tiebreak.py, then REPS rounds of
# bench.py --tiebreak exact and device (plus device under each extra env setting given as an
# argument, e.g. SHREDWORD_SELECT_TABLE_SLOTS=8388608).  Outputs gpurun_out/tb2_<label>_<r>.json/.err
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiebreak.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05_tb_tests.log 2>&1 || exit $?
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python -u bench.py --tiebreak exact --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 \
    > gpurun_out/tb2_exact_$r.json 2> gpurun_out/tb2_exact_$r.err || exit $?
  for setting in - "$@"; do
    label=device${setting#SHREDWORD_}
    [ "$setting" = "-" ] && { setting="SHREDWORD_SELECT_REPORT=1"; label=device; }
    env $setting SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python -u bench.py --tiebreak device --no-cpu-baseline \
      --encode-reps 0 --pair-count-reps 0 > gpurun_out/tb2_${label}_$r.json 2> gpurun_out/tb2_${label}_$r.err || exit $?
  done
done
echo done
