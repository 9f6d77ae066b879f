export SHREDWORD_BENCH_DIR=/dev/shm/sw
(while sleep 50; do echo hb; done) & HB=$!
rc=0
for setting in ${SETTINGS:-SHREDWORD_LOAD_READERS=16 SHREDWORD_LOAD_READERS=8}; do
  timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.'); import bench
cfg=dict(bench.CONFIGS['c5']); p=bench.corpus_path(cfg,'c5'); print('gen', bench.ensure_corpus(cfg,p))" >> gpurun_out/firstload.txt 2>&1 || { rc=1; break; }
  echo "== first load, $setting" >> gpurun_out/firstload.txt
  env ${setting//,/ } SHREDWORD_LOAD_REPORT=1 timeout -k 10 200 python3 shredword-trainer_amd/tools/load_once.py --config c5 >> gpurun_out/firstload.txt 2>&1 || { rc=1; break; }
  rm -rf /dev/shm/sw
done
rm -rf /dev/shm/sw
kill $HB
exit $rc
