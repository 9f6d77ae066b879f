#!/bin/bash
# Round-4: k_resident phase stamps at C5 100 GB (the first 2,520 merges: vocab 2776), resident only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export SHREDWORD_BENCH_DIR=/dev/shm/shredword_full
( while sleep 60; do echo "[stamps] alive $(date +%T)"; done ) &
HB=$!
timeout -k 10 900 python -u shredword-trainer_amd/tools/resident_stamps.py --config c5 --vocab 2776 \
  > gpurun_out/r04_c5_resident_stamps.log 2>&1
rc=$?
kill $HB
rm -rf /dev/shm/shredword_full
exit $rc
