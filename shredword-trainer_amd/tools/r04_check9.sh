#!/bin/bash
# Round-4 GPU check 9: the whole -m gpu suite on the current tree, then the per-merge device trace
# of the indexed loop at C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -u shredword-trainer_amd/tools/index_trace.py --config c3 --out gpurun_out/r04_index_trace_c3.npy \
  > gpurun_out/r04_index_trace_c3.log 2>&1 || exit $?
