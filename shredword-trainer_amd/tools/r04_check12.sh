#!/bin/bash
# Round-4 GPU check 12: the per-merge device trace of the indexed loop at C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python -u shredword-trainer_amd/tools/index_trace.py --config c3 --out gpurun_out/r04_index_trace_c3.npy \
  > gpurun_out/r04_index_trace_c3.log 2>&1 || exit $?
