# Round profile of bench.py on one MI355X: kernel trace + stats, then the two PMC passes
# (separate runs: FETCH_SIZE, WRITE_SIZE), all under gpurun_out/.  Summaries go to profiles/
# via tools/pmc_summary.py and tools/trace_summary.py.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --pair-count-reps 2 --no-cpu-baseline > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --pair-count-reps 2 --no-cpu-baseline > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err
