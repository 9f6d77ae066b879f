#!/bin/bash
# Builder helper (runs here, never on the GPU box): gpurun with retries while the pool has no free
# box (exit 3: nothing ran, nothing charged).  Any other exit status is final.
#   tools/gpurun_retry.sh OUT.txt TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 30); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  echo "rc=$rc attempt=$i" >> "$out"
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
