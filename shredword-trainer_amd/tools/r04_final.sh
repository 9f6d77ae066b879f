#!/bin/bash
# Round-4 final tree on the GPU: the whole -m gpu suite, smoke(), the driver's default bench line,
# and rocprofv3 kernel stats of the same bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04_final_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/r04_final_bench_under_rocprof.json 2> gpurun_out/r04_final_bench_under_rocprof.err || exit $?
echo done
