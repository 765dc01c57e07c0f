#!/bin/bash
# Per-kernel HBM traffic of a command: FETCH_SIZE and WRITE_SIZE passes (one counter block per
# rocprofv3 run) plus a kernel trace for durations. Usage: bash tools/pmc_kernels.sh TAG cmd...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- "$@" > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 || { echo pmc $c failed; exit 1; }
  i=$((i+1))
done
echo pmc ok
