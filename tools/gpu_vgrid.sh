#!/bin/bash
# weighted parity tests (default build), then probe_grid for several variant builds.
# Usage: bash tools/gpu_vgrid.sh TAG "v1 v2 ..." key=v1,v2 ...   (variant 'default' = main build)
set -o pipefail
TAG=$1; VARS=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "weighted or delta" --timeout 120 --timeout-method thread > $OUT/pytest_w.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_w.log; exit 1; }
tail -1 $OUT/pytest_w.log
for v in $VARS; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u tools/probe_grid.py 26 "$@" > $OUT/grid_$v.log 2>&1 || { echo "grid $v failed"; tail -20 $OUT/grid_$v.log; exit 1; }
  echo "== $v"; grep "ms \[" $OUT/grid_$v.log
done
