#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-p2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_partition.py -m gpu > $OUT/pytest_part.log 2>&1 || { echo part tests failed; tail -30 $OUT/pytest_part.log; exit 1; }
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
echo p2 ok
