#!/bin/bash
# Round-4 GPU check 13: tiebreak=device pair-table size A/B (default vs 4 M and 8 M slots).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
: > gpurun_out/r04_k5_table_ab.txt
for slots in 0 4194304 8388608 0; do
  SHREDWORD_SELECT_TABLE_SLOTS=$slots SHREDWORD_SELECT_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device \
    --steps 3 --warmup 1 --encode-reps 0 --pair-count-reps 0 --no-cpu-baseline > gpurun_out/k5ab.json 2> gpurun_out/k5ab.err || exit $?
  echo "slots=$slots $(python3 -c "import json;d=json.load(open('gpurun_out/k5ab.json'));t=d['tiebreak_device'];print(round(d['value']), t['table_slots'])") $(grep 'SELECT\] [0-9]* merges' gpurun_out/k5ab.err | head -1)" >> gpurun_out/r04_k5_table_ab.txt
done
