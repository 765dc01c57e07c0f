#!/bin/bash
# binned light rounds: parity first (small, then the full-size certificate), then the k26w A/B and a timeline
set -o pipefail
OUT=gpurun_out/r3h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "binned" > $OUT/tests.log 2>&1 || { echo binned tests failed; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "weighted" > $OUT/tests2.log 2>&1 || { echo weighted tests failed; tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
PASSES=2 bash tools/ab_opts.sh r3h_ab "--opt bin_min=0" "" "--opt bin_min=1000000" "--opt bin_min=16000000" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/stats_probe.py 26 2 round_log=1 > $OUT/rlog.out 2> $OUT/rlog.err || exit 1
grep -v amdgpu $OUT/rlog.err | grep -v rocprof | head -40
python3 tools/trace_solve.py $OUT/kt/run_kernel_trace.csv 0 v2_init_k > $OUT/tl0.txt; head -60 $OUT/tl0.txt
python3 tools/trace_solve.py $OUT/kt/run_kernel_trace.csv 1 v2_init_k > $OUT/tl1.txt; tail -3 $OUT/tl1.txt
