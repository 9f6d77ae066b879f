# Kernel stats + FETCH/WRITE PMC passes of the load and encode legs (bench --steps 1, no K1 leg;
# CFG=c2|c3, default c3).
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
A="--config ${CFG:-c3} --steps 1 --warmup 0 --pair-count-reps 0 --encode-reps 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/elp_stats -o run --output-format csv -- python3 bench.py $A > gpurun_out/elp_stats.json 2> gpurun_out/elp_stats.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/elp_$c -o run --output-format csv -- python3 bench.py $A > gpurun_out/elp_$c.json 2> gpurun_out/elp_$c.err
done
echo done
