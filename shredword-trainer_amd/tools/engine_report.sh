# Engine wait split (guessed vs posted merges) for the bench configs under a few speculation depths.
set -e
mkdir -p gpurun_out
for cfg in ${CFGS:-c2 c3}; do
  for d in ${DEPTHS:-1 2}; do
    SHREDWORD_ENGINE_REPORT=1 SHREDWORD_SPEC_DEPTH=$d timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline \
      --encode-reps 0 --pair-count-reps 0 --steps 2 > gpurun_out/er_${cfg}_d$d.json 2> gpurun_out/er_${cfg}_d$d.err
  done
done
echo done
