#!/bin/bash
# Round-4 GPU check 14: C3 early-guess A/B with the final defaults (helper off), 2 x 2 runs.
set -o pipefail
export TMPDIR=/tmp
REPS=3 STEPS=5 TAG=_switch bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_SWITCH_OCC=8000" "X=1" "SHREDWORD_SWITCH_OCC=2500"
