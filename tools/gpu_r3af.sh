#!/bin/bash
# round 3: kernel statistics of the weighted partition (tools/probe_wpart.py 26 at its defaults,
# world 1 and 2, 3 roots each)
set -o pipefail
OUT=gpurun_out/r3af; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 -u tools/probe_wpart.py 26 "0.1,4,0" > $OUT/kt.log 2>&1 || { echo kt failed; tail $OUT/kt.log; exit 1; }
grep world $OUT/kt.log
python3 tools/kt_summary.py $OUT/kt/run_kernel_stats.csv 1 25
echo r3af ok
