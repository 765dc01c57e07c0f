#!/bin/bash
# BFS latency experiments: tools/bfs_time.py under libpj variants and grid sizes.
set -o pipefail
OUT=gpurun_out/r2e; mkdir -p $OUT
for v in default devatom pb16 rpi8 rpi2; do
  if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
  timeout -k 10 200 python3 -u tools/bfs_time.py > $OUT/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep "direction=0" $OUT/$v.log
done
unset PJ_LIB_OVERRIDE
for gpc in 4 8; do
  timeout -k 10 200 python3 -u tools/bfs_time.py grid_per_cu=$gpc > $OUT/gpc$gpc.log 2>&1 || { echo "gpc $gpc failed"; tail -5 $OUT/gpc$gpc.log; exit 1; }
  echo "== gpc $gpc"; grep "direction=0" $OUT/gpc$gpc.log
done
