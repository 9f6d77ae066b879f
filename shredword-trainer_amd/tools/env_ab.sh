#!/bin/bash
# bench.py under env settings, interleaved over REPS rounds on one box ("-" = the defaults):
#   REPS=2 TESTS="hybrid or index" TEST_ENV=SHREDWORD_WL_WT=1 bash shredword-trainer_amd/tools/env_ab.sh SHREDWORD_WL_WT=0 SHREDWORD_WL_WT=1
# TESTS (optional): a pytest -k expression over the -m gpu parity + sequence tests, run first under TEST_ENV.
# Outputs: gpurun_out/ab_<setting>_<r>.json / .err, gpurun_out/ab_tests.log
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  env ${TEST_ENV:-SHREDWORD_AB=1} timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sequences.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/ab_tests.log 2>&1 || exit $?
fi
for r in $(seq 1 ${REPS:-2}); do
  for setting in "$@"; do
    label=${setting//[^A-Za-z0-9_=-]/_}
    [ "$setting" = "-" ] && { setting="SHREDWORD_AB=1"; label=defaults; }
    env $setting timeout -k 10 300 python -u bench.py --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 $BENCH_ARGS \
      > gpurun_out/ab_${label}_$r.json 2> gpurun_out/ab_${label}_$r.err || exit $?
  done
done
echo done
