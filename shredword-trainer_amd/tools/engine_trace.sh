# Per-merge host timings (select / launch / wait / apply, records, guess hit) of one C3 train():
# bench --steps 1 with SHREDWORD_ENGINE_TRACE; the last train() wins the file.  TAG=<suffix> names the outputs.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SHREDWORD_ENGINE_TRACE=gpurun_out/engine_trace_${CFG:-c3}${TAG}.txt SHREDWORD_ENGINE_REPORT=1 timeout -k 10 400 \
  python -u bench.py --config ${CFG:-c3} --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 --steps 1 --warmup 1 $EXTRA \
  > gpurun_out/et_${CFG:-c3}${TAG}.json 2> gpurun_out/et_${CFG:-c3}${TAG}.err
echo done
