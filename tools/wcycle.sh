#!/bin/bash
# weighted-solver cycle: weighted parity tests, then the k26w bench line twice (spread)
set -o pipefail
TAG=${1:-w}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "weighted or delta" tests/test_multisource.py tests/test_partition.py > $OUT/pytest_gpu.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 32 --warmup 4 "$@" > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo bench failed; tail -5 $OUT/bench$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench$i.json').read().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['kernel_ms_mean'], d['roofline']['frac'])"
done
