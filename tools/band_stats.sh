#!/bin/bash
# Per-round statistics of k26w solves (PJ_V2_STATS build) and the per-band workload (host CSR):
# bash tools/band_stats.sh TAG [scale] [delta]
set -o pipefail
TAG=${1:-bands}; SCALE=${2:-26}; DELTA=${3:-14}; OUT=gpurun_out/$TAG; mkdir -p $OUT
PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/stats/libpj.so timeout -k 10 200 python3 -u tools/traffic_probe.py $SCALE 2 1 > $OUT/stats.out 2> $OUT/stats.err || { tail -5 $OUT/stats.err; exit 1; }
grep -c band $OUT/stats.err
timeout -k 10 400 python3 -u tools/probe_bands.py $SCALE $DELTA 1 > $OUT/bands.txt 2>&1 || { tail -5 $OUT/bands.txt; exit 1; }
head -40 $OUT/bands.txt
