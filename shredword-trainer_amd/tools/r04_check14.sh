#!/bin/bash
# Round-4 GPU check 14: C3 early-guess A/B with the final defaults (helper off), 2 x 2 runs.
set -o pipefail
export TMPDIR=/tmp
REPS=3 STEPS=5 TAG=_pin bash shredword-trainer_amd/tools/ab.sh "SHREDWORD_PIN_EXCLUSIVE=0" "SHREDWORD_PIN_EXCLUSIVE=1"
