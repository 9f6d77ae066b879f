#!/bin/bash
# Round-4: the whole -m gpu suite and smoke() on the final tree (after the gather fallback and the window knob).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04_final4_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final4_smoke.log 2>&1 || exit $?
echo done
