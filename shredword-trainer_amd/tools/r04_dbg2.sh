#!/bin/bash
# Debug: test_argmax_verifier on the stream layout under early guess / apply helper on and off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
: > gpurun_out/r04_dbg2.log
for env in "X=1" "SHREDWORD_EARLY_GUESS=0" "SHREDWORD_APPLY_HELPER=0" "SHREDWORD_EARLY_GUESS=0 SHREDWORD_APPLY_HELPER=0"; do
  echo "== $env" >> gpurun_out/r04_dbg2.log
  env $env timeout -k 10 200 python -u -m pytest "tests/test_gpu_parity.py::test_argmax_verifier" -k "stream" -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED" >> gpurun_out/r04_dbg2.log
  true
done
