#!/bin/bash
set -o pipefail
TAG=${1:-w2}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python tools/probe_weighted.py 26 8 16 32 64 128 > $OUT/dsweep26.log 2>&1 || { echo sweep failed; tail $OUT/dsweep26.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/probe_weighted_scales.py 26 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
echo w2 ok
