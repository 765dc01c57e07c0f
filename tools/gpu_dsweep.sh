#!/bin/bash
set -o pipefail
TAG=${1:-ds}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for sc in 22 26; do
timeout -k 10 300 python tools/probe_weighted.py $sc 8 16 24 32 48 64 > $OUT/ds$sc.log 2>&1 || { echo sweep failed; tail $OUT/ds$sc.log; exit 1; }
done
echo ds ok
