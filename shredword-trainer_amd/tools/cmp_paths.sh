# Merge-loop paths side by side on the bench configs: hybrid (default; SWITCH=occurrences list),
# indexed only, resident only.
set -e
mkdir -p gpurun_out
for cfg in ${CFGS:-c2 c3}; do
  for mode in ${MODES:-hybrid index resident}; do
    for sw in ${SWITCH:-2048}; do
      case $mode in
        hybrid) env="SHREDWORD_HYBRID=1 SHREDWORD_INDEX=1 SHREDWORD_SWITCH_OCC=$sw" ;;
        index) env="SHREDWORD_HYBRID=0 SHREDWORD_INDEX=1" ;;
        resident) env="SHREDWORD_HYBRID=0 SHREDWORD_INDEX=0" ;;
      esac
      env $env timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --encode-reps 0 --pair-count-reps 0 --steps ${STEPS:-3} > gpurun_out/cmp_${cfg}_${mode}_${sw}.json 2> gpurun_out/cmp_${cfg}_${mode}_${sw}.err
      [ "$mode" = hybrid ] || break
    done
  done
done
echo done
