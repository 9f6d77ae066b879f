#!/bin/bash
# The streamed load's file -> HBM rate under reader settings: CFG's corpus in /dev/shm, one
# load_corpus per setting (tools/load_once.py with SHREDWORD_LOAD_REPORT=1), REPS rounds; the
# [LOAD] lines go to gpurun_out/load_sweep_$CFG.txt.
#   CFG=c3 REPS=2 bash shredword-trainer_amd/tools/load_sweep.sh "SHREDWORD_LOAD_READERS=8" "SHREDWORD_LOAD_READERS=16"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c3}
REPS=${REPS:-2}
export SHREDWORD_BENCH_DIR=/dev/shm/shredword_sweep
OUT=gpurun_out/load_sweep_${CFG}${TAG}.txt
: > $OUT
timeout -k 10 600 python3 shredword-trainer_amd/tools/load_once.py --config $CFG > /dev/null 2>&1 || exit $?  # the corpus
for r in $(seq 1 $REPS); do
  for setting in "$@"; do
    echo "== $setting" >> $OUT
    env $setting SHREDWORD_LOAD_REPORT=1 timeout -k 10 300 python3 shredword-trainer_amd/tools/load_once.py --config $CFG \
      > gpurun_out/load_sweep_run.txt 2>&1 || { cat gpurun_out/load_sweep_run.txt >> $OUT; exit 1; }
    grep -E "\[LOAD\] phase (file_to_hbm|word_table)|: load " gpurun_out/load_sweep_run.txt >> $OUT
  done
done
rm -rf /dev/shm/shredword_sweep
echo done
