#!/bin/bash
set -o pipefail
OUT=gpurun_out/c2; mkdir -p $OUT
timeout -k 10 240 python tools/probe_weighted_scales.py 22 24 > $OUT/w2224.log 2>&1 || { echo w2224 failed; tail $OUT/w2224.log; exit 1; }
timeout -k 10 120 python tools/probe_workloads.py > $OUT/wl.log 2>&1 || echo "workloads failed (continuing)"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 tools/traffic_probe.py 22 8 > $OUT/pmc_$c.log 2>&1 || { echo pmc $c failed; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/traffic_probe.py 22 8 > $OUT/kt.log 2>&1 || { echo kt failed; exit 1; }
timeout -k 10 400 python tools/probe_weighted_scales.py 26 > $OUT/w26.log 2>&1 || { echo w26 failed; tail $OUT/w26.log; exit 1; }
echo c2 ok
