# GPU check of the load and encode paths: their tests, then a C3 bench line (SHREDWORD_LOAD_REPORT on).
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_api.py -k "word_count or encode or Encode" > gpurun_out/t_enc.log 2>&1
SHREDWORD_LOAD_REPORT=1 timeout -k 10 500 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_c3b.json 2> gpurun_out/bench_c3b.err
echo ok
