#!/bin/bash
# round 3: light pull rounds of the weighted partition: partition tests, probe (s24w, s26w)

set -o pipefail
OUT=gpurun_out/r3s; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_gpu_parity.py -k "wpart or weighted_s22 or partition or cli_processes or multi" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/probe_wpart.py 24 > $OUT/wpart24.log 2>&1 || { echo probe24 failed; tail $OUT/wpart24.log; exit 1; }
grep world $OUT/wpart24.log
timeout -k 10 400 python -u tools/probe_wpart.py 26 > $OUT/wpart26.log 2>&1 || { echo probe26 failed; tail $OUT/wpart26.log; exit 1; }
grep world $OUT/wpart26.log
