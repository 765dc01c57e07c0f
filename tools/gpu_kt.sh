#!/bin/bash
# kernel trace of one command: bash tools/gpu_kt.sh TAG cmd...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- "$@" > $OUT/kt.log 2>&1 || { echo kt failed; tail $OUT/kt.log; exit 1; }
echo kt ok
