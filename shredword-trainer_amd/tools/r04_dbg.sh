#!/bin/bash
# Debug: tiebreak=device cases with the host phase, first trace difference against the oracle rule.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
make -s -C oracle port > /dev/null
for c in small_v300 ascii1m_unk7_cov09 utf8_2m_v2000_mpf50 mixed2m_v4000; do
  SHREDWORD_SELECT_REPORT=1 SHREDWORD_RESIDENT_REPORT=1 timeout -k 10 120 python -u shredword-trainer_amd/tools/tiebreak_debug.py $c 50 \
    >> gpurun_out/r04_dbg.log 2>&1 || { echo "rc=$? on $c" >> gpurun_out/r04_dbg.log; exit 1; }
done
