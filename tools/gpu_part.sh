#!/bin/bash
# Partitioned BFS on the GPU box: parity tests (world 1, world 2 sharing the GPU), then timing probes.
set -o pipefail
OUT=gpurun_out/${1:-part}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_partition.py -m gpu > $OUT/pytest_part.log 2>&1 || { echo part tests failed; tail -30 $OUT/pytest_part.log; exit 1; }
timeout -k 10 120 python -u tools/probe_part.py 22 4 --single > $OUT/probe22.log 2>&1 || { echo probe22 failed; tail -20 $OUT/probe22.log; exit 1; }
timeout -k 10 200 python -u tools/probe_part.py 26 3 > $OUT/probe26.log 2>&1 || { echo probe26 failed; tail -20 $OUT/probe26.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_all.log 2>&1 || { echo full gpu tests failed; tail -30 $OUT/pytest_all.log; exit 1; }
echo part ok
