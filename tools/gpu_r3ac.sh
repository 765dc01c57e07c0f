#!/bin/bash
# round 3: weighted partition light rounds count their new frontier per block (one atomic per
# block, was one per marked vertex on one word) and the band select takes one atomicMin per
# block: partition tests, then tools/probe_wpart.py at s24w and s26w (world 1 and 2)
set -o pipefail
OUT=gpurun_out/r3ac; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_tree.py tests/test_gpu_parity.py -k "wpart or partition or weighted_s22 or cli_processes or multi or tree" > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/probe_wpart.py 24 > $OUT/wpart24.log 2>&1 || { echo probe24 failed; tail $OUT/wpart24.log; exit 1; }
grep world $OUT/wpart24.log
timeout -k 10 400 python -u tools/probe_wpart.py 26 > $OUT/wpart26.log 2>&1 || { echo probe26 failed; tail $OUT/wpart26.log; exit 1; }
grep world $OUT/wpart26.log
echo r3ac ok
