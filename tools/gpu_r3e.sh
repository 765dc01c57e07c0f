#!/bin/bash
# kernel timeline of the two stats_probe solves with the round log beside it
set -o pipefail
OUT=gpurun_out/r3e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/stats_probe.py 26 2 round_log=1 > $OUT/rlog.out 2> $OUT/rlog.err || { echo failed; tail -5 $OUT/rlog.err; exit 1; }
grep -v amdgpu $OUT/rlog.err | grep -v rocprof
python3 tools/trace_solve.py $OUT/kt/run_kernel_trace.csv 0 v2_init_k
python3 tools/trace_solve.py $OUT/kt/run_kernel_trace.csv 1 v2_init_k
