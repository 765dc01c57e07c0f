#!/bin/bash
# Standard GPU-box cycle: parity tests, a short bench, then a rocprofv3 kernel trace.
# Usage (on the box, from the repo root): bash tools/gpu_cycle.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline "$@" > "$OUT/prof_bench.log" 2>&1 || { echo "rocprof failed"; exit 1; }
echo "cycle ok"
