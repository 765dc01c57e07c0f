#!/bin/bash
# Kernel trace of k26w solves (tools/traffic_probe.py 26 4 1) and the per-sync segments of one solve.
# Usage: bash tools/solve_trace.sh [TAG]
set -o pipefail
OUT=gpurun_out/${1:-solve}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 tools/traffic_probe.py 26 4 1 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
python3 tools/trace_bands.py $OUT/kt/kt_kernel_trace.csv -2 v2_source_k
