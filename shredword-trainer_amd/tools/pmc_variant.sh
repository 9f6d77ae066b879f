# FETCH_SIZE / WRITE_SIZE passes (separate runs) of one bench step of a library build:
#   LIB=variants/libtrainer_X.so TAG=_x bash shredword-trainer_amd/tools/pmc_variant.sh
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  SHREDWORD_LIB=${LIB:-shredword-trainer_amd/shredword/libtrainer.so} timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/pmc${TAG}_${c} -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --pair-count-reps 0 --encode-reps 0 --no-cpu-baseline --device-leg-steps 0 \
    > gpurun_out/pmc${TAG}_${c}.json 2> gpurun_out/pmc${TAG}_${c}.err
done
echo done
