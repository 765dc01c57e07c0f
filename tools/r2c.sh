#!/bin/bash
# ingestion cycle: ingestion + parity tests, then the CLI phase probe under a kernel trace
set -o pipefail
OUT=gpurun_out/r2c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ingest.py tests/test_gpu_parity.py > $OUT/pytest_gpu.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/ingest_probe.py 22 > $OUT/ingest.log 2>&1 || { echo probe failed; tail -20 $OUT/ingest.log; exit 1; }
cat $OUT/ingest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/ingest_probe.py 22 > $OUT/kt.log 2>&1 || { echo kt failed; tail $OUT/kt.log; exit 1; }
echo cycle ok
