#!/bin/bash
# The load's phase report (SHREDWORD_LOAD_REPORT=1) on CFGS' corpora in /dev/shm, REPS loads per
# setting (each setting is an env assignment, or "-" for the defaults), one process per load:
#   CFGS="c3 c5" REPS=2 bash shredword-trainer_amd/tools/load_phases.sh - SHREDWORD_LOAD_EVICT=75
# Output: gpurun_out/load_phases_<cfg><TAG>.txt
export SHREDWORD_BENCH_DIR=/dev/shm/sw
[ $# -eq 0 ] && set -- -
(while sleep 50; do echo hb; done) & HB=$!
rc=0
for c in ${CFGS:-c3 c5}; do
  timeout -k 10 300 python3 shredword-trainer_amd/tools/load_once.py --config $c > /dev/null 2>&1 || { rc=1; break; }
  for r in $(seq 1 ${REPS:-2}); do
    for setting in "$@"; do
      [ "$setting" = "-" ] && setting="SHREDWORD_LOAD_REPORT=1"
      echo "== $setting" >> gpurun_out/load_phases_${c}${TAG}.txt
      env $setting SHREDWORD_LOAD_REPORT=1 timeout -k 10 200 python3 shredword-trainer_amd/tools/load_once.py \
        --config $c >> gpurun_out/load_phases_${c}${TAG}.txt 2>&1 || { rc=1; break 3; }
    done
  done
  rm -rf /dev/shm/sw
done
rm -rf /dev/shm/sw
kill $HB
exit $rc
