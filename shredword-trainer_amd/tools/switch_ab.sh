#!/bin/bash
# C3 bench under hybrid switch settings (SHREDWORD_SWITCH_OCC: the resident loop hands over once a
# window of merges changed fewer table entries than this), REPS rounds; then the C5 100 GB sweep.
#   bash shredword-trainer_amd/tools/switch_ab.sh 2000 4000 8000
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for occ in "$@"; do
    SHREDWORD_SWITCH_OCC=$occ timeout -k 10 300 python -u bench.py --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 \
      > gpurun_out/sw_c3_${occ}_$r.json 2> gpurun_out/sw_c3_${occ}_$r.err || exit $?
  done
done
[ -n "$C5" ] || exit 0
timeout -k 10 800 python -u shredword-trainer_amd/tools/c5_switch_sweep.py --occ "$@" --out gpurun_out/r05_c5_switch_sweep.json \
  > gpurun_out/r05_c5_switch_sweep.log 2>&1
rc=$?
rm -rf /dev/shm/shredword_full
exit $rc
