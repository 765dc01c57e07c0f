#!/bin/bash
# Quick cycle for the weighted solver: weighted parity tests, scale probe, kernel-trace stats of the bench line.
set -o pipefail
TAG=${1:-q}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "weighted or kronecker_generator" > $OUT/pytest_w.log 2>&1 || { echo weighted tests failed; tail -30 $OUT/pytest_w.log; exit 1; }
timeout -k 10 200 python -u tools/probe_weighted_scales.py 26 > $OUT/wscales.log 2>&1 || { echo probe failed; tail -20 $OUT/wscales.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/kt.log 2>&1 || { echo kt failed; tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 200 python -u tools/probe_weighted.py 26 8 12 16 32 > $OUT/dsweep.log 2>&1 || { echo dsweep failed; exit 1; }
echo quick ok
