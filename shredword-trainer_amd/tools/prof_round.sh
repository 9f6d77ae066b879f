# Round profile of bench.py (default config) on one MI355X: kernel trace + stats, then the two
# PMC passes (separate runs: FETCH_SIZE, WRITE_SIZE), all under gpurun_out/.  Summaries go to
# profiles/ via tools/pmc_summary.py and tools/prof_summary.py.
#   CFG=c3 bash shredword-trainer_amd/tools/prof_round.sh
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-c3}
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- \
  python3 bench.py --config $CFG > gpurun_out/prof_bench_$CFG.json 2> gpurun_out/prof_bench_$CFG.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_$CFG -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 1 --warmup 0 --pair-count-reps 2 --encode-reps 1 --no-cpu-baseline \
    > gpurun_out/pmc_${c}_$CFG.json 2> gpurun_out/pmc_${c}_$CFG.err
done
echo done
