#!/bin/bash
# configs[0] (web-Google-shaped) BFS direction-switch sweep: bash tools/gpu_wg_sweep.sh TAG "opts" ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; i=0
for o in "$@"; do
  timeout -k 10 120 python bench.py --workload wg --steps 64 --warmup 4 --no-cpu-baseline --no-secondary --no-partitioned $o > "$OUT/wg_$i.log" 2>&1 || { echo "variant $i failed"; tail -5 "$OUT/wg_$i.log"; exit 1; }
  echo "[$o] $(tail -1 "$OUT/wg_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_mean"], d["bands_or_levels"])')"
  i=$((i+1))
done
