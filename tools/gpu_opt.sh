#!/bin/bash
# Option sweep + kernel trace of the bench under given --opt settings.
# Usage: bash tools/gpu_opt.sh TAG "KEY v1 v2 ..." [bench --opt args...]
set -o pipefail
TAG=$1; SWEEP=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u tools/probe_opt.py 26 $SWEEP > $OUT/sweep.log 2>&1 || { echo sweep failed; tail -20 $OUT/sweep.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --steps 8 --warmup 1 "$@" > $OUT/kt.log 2>&1 || { echo kt failed; tail -20 $OUT/kt.log; exit 1; }
cat $OUT/sweep.log
echo opt ok
