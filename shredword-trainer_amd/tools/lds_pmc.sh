# LDS counters of the merge loops on one bench config (k_resident's early merges: delta-hash
# contention vs bank conflicts vs HBM waits), one rocprofv3 --pmc pass of 8 SQ counters over a
# one-step bench, plus the per-merge index trace and engine trace of the same config.
#   CFG=c3 bash shredword-trainer_amd/tools/lds_pmc.sh
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${CFG:-c3}
TAG=${TAG:-}
timeout -k 10 300 python -u shredword-trainer_amd/tools/index_trace.py --config $CFG --out gpurun_out/index_trace_$CFG$TAG.npy \
  > gpurun_out/index_trace_$CFG$TAG.json 2> gpurun_out/index_trace_$CFG$TAG.err
SHREDWORD_ENGINE_TRACE=gpurun_out/engine_trace_$CFG$TAG.txt SHREDWORD_ENGINE_REPORT=1 timeout -k 10 300 \
  python -u bench.py --config $CFG --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 --steps 1 --warmup 1 \
  > gpurun_out/et_$CFG$TAG.json 2> gpurun_out/et_$CFG$TAG.err
if [ -z "$NO_PMC" ]; then
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_lds_$CFG$TAG -o run \
    --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 0 --pair-count-reps 0 --encode-reps 0 \
    --no-cpu-baseline > gpurun_out/pmc_lds_$CFG$TAG.json 2> gpurun_out/pmc_lds_$CFG$TAG.err
fi
echo done
