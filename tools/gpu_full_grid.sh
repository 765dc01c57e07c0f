#!/bin/bash
# all gpu tests, then a weighted s26 grid sweep. Usage: bash tools/gpu_full_grid.sh TAG key=v1,v2 ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python -u tools/probe_grid.py 26 "$@" > $OUT/grid.log 2>&1 || { echo grid failed; tail -20 $OUT/grid.log; exit 1; }
cat $OUT/grid.log
