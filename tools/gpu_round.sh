#!/bin/bash
# Full round cycle on the GPU box: all gpu tests, the default bench line, its kernel trace, PMC traffic.
set -o pipefail
TAG=${1:-round}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 500 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 tools/traffic_probe.py 26 4 1 > $OUT/pmc_$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
echo round cycle ok
