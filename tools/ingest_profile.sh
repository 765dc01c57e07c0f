#!/bin/bash
# Ingestion profile: CLI phase times (ingest_probe), kernel traces of the CLI on the K22 and WG text,
# and FETCH_SIZE / WRITE_SIZE passes (one counter group per run) on the K22 CLI run.
set -o pipefail
OUT=gpurun_out/${1:-ingest}; mkdir -p $OUT
export PJ_SCRATCH=/tmp
timeout -k 10 300 python -u tools/ingest_probe.py 22 --keep > $OUT/ingest.log 2>&1 || { echo probe failed; tail -20 $OUT/ingest.log; exit 1; }
grep -v amdgpu $OUT/ingest.log
K22=$(grep "kept .*k22.txt" $OUT/ingest.log | awk '{print $3}')
WG=$(grep "kept .*wg.txt" $OUT/ingest.log | awk '{print $3}')
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PJ_PHASES=1
for t in "22 $K22 1" "wg $WG 0"; do
  set -- $t
  mkdir -p $OUT/ing$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ing$1/kt -o run -- paralleljohnson_amd/bin/parallel_johnson $2 $3 /tmp/sol.txt > $OUT/ing$1/kt.log 2>&1 || { echo kt failed; tail $OUT/ing$1/kt.log; exit 1; }
  grep -E "phase|Time" $OUT/ing$1/kt.log
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/ing22/p$c -o run -- paralleljohnson_amd/bin/parallel_johnson $K22 1 /tmp/sol.txt > $OUT/ing22/p$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
python3 tools/pmc_kernel_table.py $OUT/ing22
rm -f $K22 $WG /tmp/sol.txt
echo ingest profile ok
