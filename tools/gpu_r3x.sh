#!/bin/bash
# round 3: per-round log (round_log: kind, frontier, its light edges) of k26w solves beside their
# kernel trace, to map the light rounds' time to their frontiers
set -o pipefail
OUT=gpurun_out/r3x; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/stats_probe.py 26 3 round_log=1 > $OUT/rl.out 2> $OUT/rl.err || { echo kt failed; tail $OUT/rl.err; exit 1; }
grep -c round $OUT/rl.err
echo r3x ok
