#!/bin/bash
# BFS grid / pull-variant timing (direction auto, small levels on)
set -o pipefail
OUT=gpurun_out/r2g; mkdir -p $OUT
run() { timeout -k 10 120 python3 -u tools/bfs_time.py dirs=0 smalls=1 "$@" 2>&1 | grep -v amdgpu | grep direction; }
for gpc in 2 3 4; do
  run grid_per_cu=$gpc pull_stream=0 && run grid_per_cu=$gpc pull_stream=1 || exit 1
done
export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/rpi2/libpj.so
for gpc in 2 3; do run grid_per_cu=$gpc pull_stream=0 || exit 1; done
export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/rpi1/libpj.so
for gpc in 2 3; do run grid_per_cu=$gpc pull_stream=0 || exit 1; done
