# A/B of environment settings on one box: bench.py (timed steps only) alternating between the
# settings given as arguments, each REPS times; one line per run with the setting and the value.
#   CFG=c3 REPS=2 bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_WL_WT=0" "SHREDWORD_WL_WT=1"
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${CFG:-c3}
REPS=${REPS:-2}
STEPS=${STEPS:-5}
OUT=gpurun_out/ab_${CFG}${TAG}.txt
: > $OUT
for r in $(seq 1 $REPS); do
  for setting in "$@"; do
    env $setting timeout -k 10 300 python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline \
      --encode-reps 0 --pair-count-reps 0 > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_run.json')); ml=d['merge_loop']; \
ix=ml.get('index',{}); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],1), \
'parity', all(d.get('parity_fullsize',{'x':True}).values() if isinstance(d.get('parity_fullsize'),dict) else [True]), \
'idx_dev_us', round(ix.get('device_busy_us_per_merge',0),2), 'post_flag', round(ix.get('host_post_to_flag_us_per_merge',0),2), \
'host', {k: round(v,3) for k,v in ml['host_s'].items()})" "$setting" | tee -a $OUT
  done
done
echo done
