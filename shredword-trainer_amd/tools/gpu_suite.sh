#!/bin/bash
# The whole -m gpu suite and smoke() on one MI355X, as the driver runs them at round end.
#   TAG=r05_final bash shredword-trainer_amd/tools/gpu_suite.sh   (logs: gpurun_out/$TAG_*.log)
# Extra pytest arguments go in PYTEST_ARGS (e.g. -k "not full_size").  Each GPU step has its own
# time limit and the steps are chained: a failed step ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
TAG=${TAG:-suite}
export SHREDWORD_HEARTBEAT_FILE=gpurun_out/${TAG}_heartbeat.log
timeout -k 10 ${SUITE_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  $PYTEST_ARGS > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
echo done
