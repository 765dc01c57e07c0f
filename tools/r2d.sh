#!/bin/bash
# kernel trace of the CLI itself on the K22 and WG text (ingestion kernels)
set -o pipefail
OUT=gpurun_out/r2d; mkdir -p $OUT
export PJ_SCRATCH=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ingest.py tests/test_gpu_parity.py tests/test_csr_cache.py > $OUT/pytest_gpu.log 2>&1 || { echo tests failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/ingest_probe.py 22 --keep > $OUT/ingest.log 2>&1 || { echo probe failed; tail -20 $OUT/ingest.log; exit 1; }
cat $OUT/ingest.log
K22=$(grep "kept .*k22.txt" $OUT/ingest.log | awk '{print $3}')
WG=$(grep "kept .*wg.txt" $OUT/ingest.log | awk '{print $3}')
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt22 -o run -- paralleljohnson_amd/bin/parallel_johnson $K22 1 /tmp/sol22.txt > $OUT/kt22.log 2>&1 || { echo kt failed; tail $OUT/kt22.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktwg -o run -- paralleljohnson_amd/bin/parallel_johnson $WG 0 /tmp/solwg.txt > $OUT/ktwg.log 2>&1 || { echo kt failed; tail $OUT/ktwg.log; exit 1; }
rm -f $K22 $WG /tmp/sol22.txt /tmp/solwg.txt
echo cycle ok
