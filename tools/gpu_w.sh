#!/bin/bash
# weighted-path cycle: weighted parity tests, scale probe, kernel trace of s22w
set -o pipefail
TAG=${1:-w}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "weighted or delta" --timeout 120 --timeout-method thread > $OUT/pytest_w.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_w.log; exit 1; }
timeout -k 10 300 python tools/probe_weighted_scales.py 22 24 26 > $OUT/wscales.log 2>&1 || { echo probe failed; tail $OUT/wscales.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/probe_weighted_scales.py 22 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
echo w ok
