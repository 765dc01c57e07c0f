#!/bin/bash
# MS1024 per-kernel time and PMC bytes: a kernel trace and FETCH_SIZE / WRITE_SIZE passes of
# tools/ms_pmc_probe.py, summarised by tools/pmc_kernel_table.py. Usage: [MS_STREAMS=1] bash tools/ms_profile.sh [TAG]
set -o pipefail
OUT=gpurun_out/${1:-ms}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/ms_pmc_probe.py 2 ${MS_STREAMS:-2} > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/p$c -o run -- python3 tools/ms_pmc_probe.py 2 ${MS_STREAMS:-2} > $OUT/p$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
python3 tools/pmc_kernel_table.py $OUT
