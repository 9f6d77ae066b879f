#!/bin/bash
# Round-4 GPU check 10: the whole -m gpu suite (early guess gated to backends holding 2 guesses),
# then an A/B of the word loop's prefetch (variants/libtrainer_nopf.so = the old load order).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04_gpu_suite2.log 2>&1 || exit $?
REPS=2 STEPS=5 TAG=_prefetch bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_LIB=$PWD/variants/libtrainer_nopf.so" "X=1"
