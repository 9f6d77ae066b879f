#!/bin/bash
# Round-4 profiles (C3, one GPU): rocprofv3 kernel trace + stats of the default bench, the two PMC
# passes (FETCH_SIZE, WRITE_SIZE; separate runs), and the per-merge host phases of one train().
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config c3 > gpurun_out/prof_bench_c3.json 2> gpurun_out/prof_bench_c3.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_c3 -o run --output-format csv -- \
    python3 bench.py --config c3 --steps 1 --warmup 0 --pair-count-reps 2 --encode-reps 1 --no-cpu-baseline \
    > gpurun_out/pmc_${c}_c3.json 2> gpurun_out/pmc_${c}_c3.err || exit $?
done
SHREDWORD_ENGINE_TRACE=gpurun_out/r04_c3_engine_trace.txt timeout -k 10 300 python3 bench.py --config c3 --steps 1 \
  --warmup 0 --pair-count-reps 0 --encode-reps 0 --no-cpu-baseline > gpurun_out/r04_c3_trace_bench.json \
  2> gpurun_out/r04_c3_trace_bench.err || exit $?
echo done
