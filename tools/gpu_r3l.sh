#!/bin/bash
# round 3: edge-tiled MS-BFS pull levels (ms_tile): batch / multi-source parity tests, an interleaved
# MS1024 timing of ms_tile 1 / 0, the MS1024 per-kernel profile (tile default)
set -o pipefail
OUT=gpurun_out/r3l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_multisource.py tests/test_csr_cache.py tests/test_partition.py -k "msbfs or multi or batch or ms1024" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/probe_ms.py "" "ms_tile=0" "ms_width=16" > $OUT/probe.log 2>&1 || { echo probe failed; tail $OUT/probe.log; exit 1; }
grep pass $OUT/probe.log
bash tools/ms_profile.sh r3l_ms > $OUT/ms.log 2>&1 || { echo ms failed; tail $OUT/ms.log; exit 1; }
tail -22 $OUT/ms.log
