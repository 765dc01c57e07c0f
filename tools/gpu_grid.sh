#!/bin/bash
# weighted parity tests, then a grid sweep at s26. Usage: bash tools/gpu_grid.sh TAG key=v1,v2 ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "weighted or delta" --timeout 120 --timeout-method thread > $OUT/pytest_w.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_w.log; exit 1; }
tail -1 $OUT/pytest_w.log
timeout -k 10 400 python -u tools/probe_grid.py 26 "$@" > $OUT/grid.log 2>&1 || { echo grid failed; tail -20 $OUT/grid.log; exit 1; }
cat $OUT/grid.log
