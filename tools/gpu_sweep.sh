#!/bin/bash
# Bench variants in one GPU call: bash tools/gpu_sweep.sh TAG "opts1" "opts2" ...
# each opts string is passed to bench.py (e.g. "--opt grid_per_cu=2").
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
i=0
for o in "$@"; do
  timeout -k 10 200 python bench.py --steps 32 --warmup 4 --no-cpu-baseline $o > "$OUT/sweep_$i.log" 2>&1 || { echo "variant $i failed"; tail -5 "$OUT/sweep_$i.log"; exit 1; }
  echo "[$o] $(tail -1 "$OUT/sweep_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms_mean"], d["levels_td_bu"])')"
  i=$((i+1))
done
