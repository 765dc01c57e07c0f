#!/bin/bash
# GPU tests of selected files (or all): bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -25 $OUT/pytest_gpu.log
exit $rc
