#!/bin/bash
# round 3: the weighted partition's light-pull threshold after the per-block frontier counts
# (push rounds got cheaper): light_pull 0 / 1.5 / 3 / 6 at s26w and s24w, world 1 and 2, twice
set -o pipefail
OUT=gpurun_out/r3ad; mkdir -p $OUT
S="0.1,4,3;0.1,4,0;0.1,4,1.5;0.1,4,6;0.1,4,3;0.1,4,0;0.1,4,1.5;0.1,4,6"
timeout -k 10 400 python -u tools/probe_wpart.py 26 "$S" > $OUT/wpart26.log 2>&1 || { echo probe26 failed; tail $OUT/wpart26.log; exit 1; }
grep world $OUT/wpart26.log
timeout -k 10 300 python -u tools/probe_wpart.py 24 "$S" > $OUT/wpart24.log 2>&1 || { echo probe24 failed; tail $OUT/wpart24.log; exit 1; }
grep world $OUT/wpart24.log
echo r3ad ok
