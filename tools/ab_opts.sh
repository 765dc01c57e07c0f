#!/bin/bash
# A/B of bench.py option sets on the k26w line, interleaved PASSES times:
# bash tools/ab_opts.sh TAG "opts1" "opts2" ...   (e.g. "--opt light_filter=0")
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for pass in $(seq 1 ${PASSES:-2}); do
  i=0
  for o in "$@"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --no-partitioned --no-tts --steps 32 --warmup 4 $o > $OUT/ab_${i}_$pass.json 2> $OUT/ab_${i}_$pass.err || { echo "[$o] failed"; tail -5 $OUT/ab_${i}_$pass.err; exit 1; }
    echo "[$o] pass $pass: $(python3 -c "import json; d=json.loads(open('$OUT/ab_${i}_$pass.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_mean'], d['roofline']['frac'])")"
    i=$((i+1))
  done
done
