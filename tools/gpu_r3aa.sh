#!/bin/bash
# round 3: kernel-argument placement (HIP_FORCE_DEV_KERNARG 0 / 1): web-Google and K22 unit
# solves (bfs_time) and the k26w line, interleaved
set -o pipefail
OUT=gpurun_out/r3aa; mkdir -p $OUT
for pass in 1 2; do
  for kv in 0 1; do
    HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python3 -u tools/bfs_time.py graphs=wg,k22 dirs=0 smalls=1 > $OUT/time_${kv}_$pass.txt 2>&1 || { tail -5 $OUT/time_${kv}_$pass.txt; exit 1; }
    echo "kernarg=$kv pass $pass: $(grep -v amdgpu $OUT/time_${kv}_$pass.txt | grep median | tr '\n' ' ')"
  done
done
for pass in 1 2; do
  for kv in 0 1; do
    HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --no-partitioned --no-tts --steps 32 --warmup 4 > $OUT/b_${kv}_$pass.json 2> $OUT/b_${kv}_$pass.err || { tail -5 $OUT/b_${kv}_$pass.err; exit 1; }
    echo "kernarg=$kv pass $pass: $(python3 -c "import json; d=json.loads(open('$OUT/b_${kv}_$pass.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_mean'])")"
  done
done
echo r3aa ok
