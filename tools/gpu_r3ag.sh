#!/bin/bash
# round 3: weighted partition keeps both light thresholds' prefixes (no per-solve recompute),
# selects 4 words per wave step, relaxes a lane's serial edges 2 per step (WP_PU; variant wpu1 = 1):
# partition tests, then probe_wpart s26w / s24w at the defaults, default and wpu1 interleaved
set -o pipefail
OUT=gpurun_out/r3ag; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_gpu_parity.py -k "wpart or partition or weighted_s22 or cli_processes or multi" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for pass in 1 2; do
  for v in default wpu1; do
    if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
    timeout -k 10 300 python -u tools/probe_wpart.py 26 "0.1,4,0" > $OUT/w26_${v}_$pass.log 2>&1 || { echo probe26 failed; tail $OUT/w26_${v}_$pass.log; exit 1; }
    echo "== $v pass $pass"; grep world $OUT/w26_${v}_$pass.log
  done
done
unset PJ_LIB_OVERRIDE
timeout -k 10 300 python -u tools/probe_wpart.py 24 "0.1,4,0;0.1,4,0" > $OUT/wpart24.log 2>&1 || { echo probe24 failed; tail $OUT/wpart24.log; exit 1; }
grep world $OUT/wpart24.log
echo r3ag ok
