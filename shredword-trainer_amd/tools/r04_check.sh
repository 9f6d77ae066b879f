#!/bin/bash
# Round-4 GPU check (run by gpurun from the repo root): the new tests, then quick C3 bench lines
# (exact and tiebreak=device) with the load phase report.  Each step has its own time limit; the
# first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sequences.py tests/test_gpu_tiebreak.py \
  "tests/test_gpu_api.py::test_file_streamed_to_hbm_matches_host" "tests/test_gpu_api.py::test_nul_byte_file_takes_the_host_path" \
  "tests/test_gpu_api.py::test_gpu_word_count_matches_host" "tests/test_gpu_api.py::test_init_and_merge_batch_abi" \
  tests/test_gpu_parity.py::test_types_layout_matches_reference tests/test_gpu_parity.py::test_index_loop_matches_reference \
  tests/test_gpu_encode.py \
  -v --maxfail=10 --timeout 240 --timeout-method thread > gpurun_out/r04_tests.log 2>&1 || exit $?
SHREDWORD_LOAD_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --encode-reps 3 --pair-count-reps 0 \
  --no-cpu-baseline > gpurun_out/r04_c3_exact.json 2> gpurun_out/r04_c3_exact.err || exit $?
SHREDWORD_EARLY_GUESS=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --encode-reps 0 --pair-count-reps 0 \
  --no-cpu-baseline > gpurun_out/r04_c3_exact_noearly.json 2> gpurun_out/r04_c3_exact_noearly.err || exit $?
SHREDWORD_LOAD_REPORT=1 timeout -k 10 300 python bench.py --tiebreak device --steps 3 --warmup 1 --encode-reps 0 \
  --pair-count-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_device.json 2> gpurun_out/r04_c3_device.err || exit $?
