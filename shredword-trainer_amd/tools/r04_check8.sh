#!/bin/bash
# Round-4 GPU check 8: the apply helper (second host thread) -- parity tests with it on, then an
# A/B of the C3 bench line on one box (on, off, on) and the engine trace with it on.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 500 python -u -m pytest tests/test_gpu_sequences.py tests/test_gpu_parity.py::test_types_layout_matches_reference \
  tests/test_gpu_parity.py::test_index_loop_matches_reference -v --timeout 240 --timeout-method thread \
  > gpurun_out/r04_helper_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --encode-reps 0 --pair-count-reps 0 --no-cpu-baseline \
  > gpurun_out/r04_ab_on1.json 2> gpurun_out/r04_ab_on1.err || exit $?
SHREDWORD_APPLY_HELPER=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --encode-reps 0 --pair-count-reps 0 \
  --no-cpu-baseline > gpurun_out/r04_ab_off.json 2> gpurun_out/r04_ab_off.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --encode-reps 0 --pair-count-reps 0 --no-cpu-baseline \
  > gpurun_out/r04_ab_on2.json 2> gpurun_out/r04_ab_on2.err || exit $?
SHREDWORD_ENGINE_TRACE=gpurun_out/r04_c3_engine_trace_helper.txt timeout -k 10 300 python3 bench.py --config c3 --steps 1 \
  --warmup 0 --pair-count-reps 0 --encode-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_trace_helper.json \
  2> gpurun_out/r04_c3_trace_helper.err || exit $?
