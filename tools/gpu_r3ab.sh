#!/bin/bash
# round 3: band selection with V2_SELW words per wave step (default 4; variant sel1 = the
# previous one-word form) and the unlabel with 8 ids per thread step (variant ul1 = one): weighted parity tests, select kernel times (kernel trace of
# tools/stats_probe.py), then the interleaved k26w A/B
set -o pipefail
OUT=gpurun_out/r3ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "weighted or s26w or kronecker" > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/kt_variants.sh r3ab_kt "tools/stats_probe.py 26 6" sel1 ul1 default > $OUT/kt.txt 2>&1 || { cat $OUT/kt.txt; exit 1; }
grep -E "==|select|unlabel|invert|light_split" $OUT/kt.txt
PASSES=2 bash tools/ab_variants.sh r3ab_ab "bench.py --no-cpu-baseline --no-secondary --no-partitioned --no-tts --steps 32 --warmup 4" sel1 ul1 default > $OUT/ab.txt 2>&1 || { cat $OUT/ab.txt; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r3ab_ab/*.log')):
    line = [l for l in open(f) if l.startswith('{')][-1]
    d = json.loads(line); print(f.split('/')[-1], d['value'], d['ms_per_step'], d['kernel_ms_mean'], d['roofline']['frac'])
PY
echo r3ab ok
