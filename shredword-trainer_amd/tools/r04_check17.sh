#!/bin/bash
# Round-4 GPU check 17: the default bench right after the whole GPU suite (the driver's order),
# then again, with the selector's huge-page coverage reported (host_thp).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04_suite3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 > gpurun_out/r04_after_suite1.json 2> gpurun_out/r04_after_suite1.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 > gpurun_out/r04_after_suite2.json 2> gpurun_out/r04_after_suite2.err || exit $?
