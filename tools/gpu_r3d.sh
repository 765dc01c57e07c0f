#!/bin/bash
# round log of two k26w solves (kind / frontier / light edges per round), then an A/B of light_pull values
set -o pipefail
OUT=gpurun_out/r3d; mkdir -p $OUT
timeout -k 10 200 python3 -u tools/stats_probe.py 26 2 round_log=1 > $OUT/rlog.out 2> $OUT/rlog.err || { echo rlog failed; tail -5 $OUT/rlog.err; exit 1; }
cat $OUT/rlog.out; grep -v amdgpu $OUT/rlog.err
PASSES=2 bash tools/ab_opts.sh r3d_ab "" "--opt light_pull=1.5" "--opt light_pull=1" "--opt light_pull=6" "--opt light_pull=0.5" || exit 1
