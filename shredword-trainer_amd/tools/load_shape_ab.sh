# k_word_count's two workgroup shapes (SHREDWORD_LOAD_WIDE=0/1) on C3: the load tests with both,
# then per shape a timed load (tools/load_once.py, twice: the first generates the corpus) and the
# FETCH_SIZE / WRITE_SIZE passes.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export SHREDWORD_BENCH_DIR=/dev/shm/shredword_ab
T=shredword-trainer_amd/tools
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_api.py -k "word_count or sharded_load" > gpurun_out/ab_tests.log 2>&1
for W in 0 1; do
  SHREDWORD_LOAD_WIDE=$W timeout -k 10 300 python3 $T/load_once.py --config c3 > gpurun_out/ab_time_$W.log 2>&1
  SHREDWORD_LOAD_WIDE=$W timeout -k 10 300 python3 $T/load_once.py --config c3 >> gpurun_out/ab_time_$W.log 2>&1
  SHREDWORD_LOAD_WIDE=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_stats_$W -o run --output-format csv -- python3 $T/load_once.py --config c3 > gpurun_out/ab_stats_$W.log 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    SHREDWORD_LOAD_WIDE=$W timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/ab_${c}_$W -o run --output-format csv -- python3 $T/load_once.py --config c3 > gpurun_out/ab_${c}_$W.log 2>&1
  done
done
rm -rf /dev/shm/shredword_ab
echo done
