#!/bin/bash
# Round-4 GPU check 18: host loop pinned on the GPU's NUMA node vs the plain domain choice (A/B).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python3 -c "
import os, sys; sys.path.insert(0, '.')
import bench, torch
torch.cuda.set_device(0)
near = bench.gpu_numa_cpus(0)
print('gpu0 numa cpus:', sorted(near)[:8], '...', len(near) if near else None)
print('allowed:', len(os.sched_getaffinity(0)))
" > gpurun_out/r04_numa_probe.txt 2>&1 || exit $?
REPS=3 STEPS=5 TAG=_numa bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_PIN_NUMA=1" "X=1"
