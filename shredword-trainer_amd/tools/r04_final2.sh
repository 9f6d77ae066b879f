#!/bin/bash
# Round-4 final tree, after the last bench.py edits: smoke() and the driver's default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final2_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r04_final2_bench.json 2> gpurun_out/r04_final2_bench.err || exit $?
echo done
